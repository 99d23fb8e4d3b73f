"""GEMM epilogue chain vs separate elementwise kernels (device-resident):
y = relu(x @ W + b) * 0.5 + c[N] - z[M,N], x [M, 512], W [512, 512].
Run with TFA_EPI_CHAIN=0 for the unabsorbed plan (GEMM+bias+relu, then one
fused elementwise kernel for the rest)."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

from tensorframes_amd import engine, tf  # noqa: E402

M, K, N = 2_000_000, 512, 512
rng = np.random.default_rng(0)
g = tf.Graph()
with g.as_default():
    x = tf.placeholder(tf.float32, [None, K], name="x")
    z = tf.placeholder(tf.float32, [None, N], name="z")
    h = tf.nn.relu(tf.nn.bias_add(tf.matmul(x, tf.constant((rng.standard_normal((K, N)) / 22).astype(np.float32))),
                                  tf.constant(rng.standard_normal(N).astype(np.float32))))
    tf.subtract(h * 0.5 + tf.constant(rng.standard_normal(N).astype(np.float32)), z, name="y")
prog = engine.program(g.serialize(), ["y"], ["x", "z"])
dev = torch.device("cuda", 0)
xi, zi = torch.randn((M, K), device=dev), torch.randn((M, N), device=dev)
plan = prog.describe([xi, zi], True)
for _ in range(3):
    engine.run_program(prog, [xi, zi], dev)
torch.cuda.synchronize()
s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
s.record()
for _ in range(10):
    engine.run_program(prog, [xi, zi], dev)
e.record()
torch.cuda.synchronize()
ms = s.elapsed_time(e) / 10
print(json.dumps({"epi_chain": os.environ.get("TFA_EPI_CHAIN", "1"), "ms": ms,
                  "tflops": 2 * M * N * K / ms / 1e9, "plan": plan}))
