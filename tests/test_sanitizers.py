"""Host-code sanitizer coverage: the C++ GraphDef codec is
built with ASan+UBSan and fed mutated fixtures (scripts/sanitize_host.sh);
the Python codec gets the same mutation treatment. GraphDefs are untrusted
input: malformed bytes must raise, never crash or read out of bounds."""
import os
import random
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FIX = os.path.join(REPO, "tests", "fixtures")


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_cpp_codec_under_asan_ubsan(tmp_path):
    env = dict(os.environ, TMPDIR=str(tmp_path))
    r = subprocess.run([os.path.join(REPO, "scripts", "sanitize_host.sh"), "3000"], cwd=REPO, env=env,
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "no sanitizer findings" in r.stdout


def test_python_codec_rejects_mutations_cleanly():
    from tensorframes_amd.graph import proto as P
    rng = random.Random(7)
    for name in ("ref_graph.pb", "ref_graph2.pb"):
        base = open(os.path.join(FIX, name), "rb").read()
        P.parse_graphdef(base)
        for i in range(3000):
            m = bytearray(base)
            if i % 3 == 0 and m:
                for _ in range(rng.randint(1, 4)):
                    m[rng.randrange(len(m))] ^= 1 << rng.randrange(8)
            elif i % 3 == 1:
                m = m[:rng.randrange(len(m) + 1)]
            else:
                at = rng.randrange(len(m) + 1)
                m[at:at] = bytes([0xFF, 0xFF, 0xFF, 0xFF, 0x0F])
            try:
                P.parse_graphdef(bytes(m))
            except P.MalformedProtoError:
                pass
