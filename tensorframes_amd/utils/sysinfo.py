"""Which machine a benchmark line came from (host name, GPU name and UUID):
the round's numbers are compared box to box, so every JSON line says where
it was measured (bench.py, bench/configs.py, examples/read_image.py)."""
from __future__ import annotations

import socket


def box_id() -> dict:
    out = {"host": socket.gethostname()}
    try:
        import torch
        if torch.cuda.is_available():
            p = torch.cuda.get_device_properties(torch.cuda.current_device())
            out["gpu"] = p.name
            uuid = getattr(p, "uuid", None)
            if uuid is not None:
                out["gpu_uuid"] = str(uuid)
            out["gpu_arch"] = getattr(p, "gcnArchName", None)
    except Exception:  # noqa: BLE001 - identification must never fail a benchmark
        pass
    return out
