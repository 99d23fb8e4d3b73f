"""reduce_blocks through a world-size-1 RCCL group (Config.force_collectives):
for a rocprofv3 kernel trace that shows the RCCL all-reduce kernel next to
the engine's column-reduce kernel. Prints one JSON line."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import tensorframes_amd as tfs  # noqa: E402
from tensorframes_amd import tf  # noqa: E402
from tensorframes_amd.parallel import dist  # noqa: E402
from tensorframes_amd.utils.logging import metrics  # noqa: E402

dist.init(backend="nccl", force=True)
rows, dim = int(os.environ.get("ROWS", "1000000")), 1024
x = torch.randn((rows, dim), device="cuda")
df = tfs.from_columns({"x": x}, num_partitions=4).cache_on_device("cuda:0")
with tf.Graph().as_default():
    xi = tf.placeholder(tf.float32, [None, dim], name="x_input")
    s = tf.reduce_sum(xi, [0], name="x")
    for _ in range(5):
        got = tfs.reduce_blocks(s, df)
err = float(np.abs(got - x.double().sum(0).cpu().numpy()).max())
m = metrics.snapshot()
print(json.dumps({"rows": rows, "max_abs_err": err, "backend": torch.distributed.get_backend(),
                  "all_reduce_calls": m.get("collective_all_reduce", 0),
                  "all_gather_object_calls": m.get("collective_all_gather_object", 0),
                  "collective_device_ms": dist.collective_device_ms()}))
dist.shutdown()
