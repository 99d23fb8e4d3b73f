"""Loader for the native extension `tensorframes_amd._C`.

The extension (C++ runtime + HIP/gfx950 kernels) is built in-tree by
``python setup.py build_ext --inplace`` (see setup.py / __graft_entry__.build).
If it is missing it is built on first import, under a file lock so that
concurrent ranks build it once.
"""
from __future__ import annotations

import fcntl
import importlib
import os
import subprocess
import sys

import torch  # noqa: F401  (loads libc10/libtorch before the extension)

_PKG_DIR = os.path.dirname(os.path.abspath(__file__))
_REPO = os.path.dirname(_PKG_DIR)


def _built() -> bool:
    return any(f.startswith("_C.") and f.endswith(".so") for f in os.listdir(_PKG_DIR))


def build(force: bool = False, quiet: bool = True) -> None:
    """Compile the extension in place (hipcc for gfx950 + the C++ runtime)."""
    lock_path = os.path.join(_REPO, ".build.lock")
    with open(lock_path, "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        try:
            if _built() and not force:
                return
            env = dict(os.environ)
            env.setdefault("PYTORCH_ROCM_ARCH", "gfx950")
            env.setdefault("MAX_JOBS", "8")
            cmd = [sys.executable, "setup.py", "build_ext", "--inplace"]
            r = subprocess.run(cmd, cwd=_REPO, env=env, capture_output=quiet, text=True)
            if r.returncode != 0:
                msg = (r.stdout or "")[-4000:] + (r.stderr or "")[-4000:] if quiet else ""
                raise RuntimeError("building tensorframes_amd._C failed:\n" + msg)
        finally:
            fcntl.flock(lk, fcntl.LOCK_UN)


def load():
    if not _built():
        if os.environ.get("TFA_NO_AUTOBUILD") == "1":
            raise ImportError("tensorframes_amd._C is not built (run `python setup.py build_ext --inplace`)")
        build()
    return importlib.import_module("tensorframes_amd._C")


_C = load()
