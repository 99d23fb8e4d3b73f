"""aggregate over 10M rows / 100k int64 keys on a device-cached frame (for
rocprofv3 --kernel-trace --stats: the factorisation kernels, the segmented
reductions). Prints one JSON line with ms per aggregate."""
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import tf  # noqa: E402

dev = torch.device("cuda", 0)
n, nk = 10_000_000, 100_000
g = torch.Generator(device=dev).manual_seed(5)
keys = torch.randint(0, nk, (n,), device=dev, generator=g, dtype=torch.int64)
x = torch.rand((n, 4), device=dev, generator=g, dtype=torch.float64)
df = tfs.from_columns({"k": keys, "x": x}, num_partitions=4).cache_on_device(dev)
with tf.Graph().as_default():
    xi = tf.placeholder(tf.double, [None, 4], name="x_input")
    s = tf.reduce_sum(xi, [0], name="x")
    tfs.aggregate(s, df.groupBy("k")).local_blocks()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(5):
        out = tfs.aggregate(s, df.groupBy("k")).local_blocks()
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / 5
print(json.dumps({"rows": n, "keys": nk, "ms_per_aggregate": dt * 1e3, "rows_per_sec": n / dt,
                  "groups": int(next(iter(out.values())).nrows)}))
