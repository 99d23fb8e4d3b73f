"""The round-up magic-number division of csrc/kernels/hip_common.h
(make_fastdiv / fdiv), emulated bit-exactly in Python: n / d ==
(umulhi(n, m) + n) >> s for every 32-bit n and every divisor in [1, 2^31).
The implicit-GEMM conv decomposes output rows into (n, oh, ow) with it
(gemm.hip ConvGeom, conv_smallc.hip)."""
import random


def make_fastdiv(d):
    s = 0
    while (1 << s) < d:
        s += 1
    m = ((1 << 32) * ((1 << s) - d)) // d + 1
    assert 0 < m < (1 << 32) or d == 1
    return m & 0xFFFFFFFF, s


def fdiv(n, f):
    m, s = f
    hi = (n * m) >> 32  # __umulhi
    return (hi + n) >> s  # 64-bit add, then shift


def test_edges_every_small_divisor():
    for d in range(1, 4097):
        f = make_fastdiv(d)
        for n in (0, 1, d - 1, d, d + 1, 2 * d - 1, (1 << 31), (1 << 32) - 1, (1 << 32) - d,
                  ((1 << 32) - 1) // d * d, ((1 << 32) - 1) // d * d - 1):
            assert fdiv(n, f) == n // d, (n, d)


def test_random_large():
    rng = random.Random(0)
    for _ in range(100000):
        d = rng.randint(1, (1 << 31) - 1)
        n = rng.randint(0, (1 << 32) - 1)
        assert fdiv(n, make_fastdiv(d)) == n // d, (n, d)


def test_conv_dims():
    # every (OW, OH) of the Inception-v3 / VGG-16 layers at 224 and 299
    for d in (1, 2, 5, 8, 12, 17, 25, 35, 52, 54, 71, 73, 109, 111, 112, 147, 149, 224):
        f = make_fastdiv(d)
        for n in range(0, 2048 * 111 * 111, 7919):
            assert fdiv(n, f) == n // d
