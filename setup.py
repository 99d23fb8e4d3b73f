"""Build the tensorframes_amd native extension (`tensorframes_amd._C`) for gfx950.

    python setup.py build_ext --inplace

Two stages, no hipify anywhere:
  1. every csrc/kernels/*.hip is compiled by hipcc for --offload-arch=gfx950
     into a position-independent object (build/hip/*.o, rebuilt when stale);
  2. the C++ runtime (GraphDef codec, IR, planner/executor, pybind11 bindings)
     is compiled as a torch C++ extension and linked with those objects and the
     HIP runtime.
"""
import glob
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

from setuptools import find_packages, setup

os.environ.setdefault("PYTORCH_ROCM_ARCH", "gfx950")

from torch.utils.cpp_extension import BuildExtension, CppExtension  # noqa: E402
import torch  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROCM = os.environ.get("ROCM_PATH", "/opt/rocm")
HIP_OBJ_DIR = os.path.join(HERE, "build", "hip")
ARCH = "gfx950"

HIP_FLAGS = [
    "-O3",
    "-std=c++17",
    f"--offload-arch={ARCH}",
    "-fPIC",
    "-ffp-contract=fast-honor-pragmas",  # contraction on, except where a kernel turns it off
    "-munsafe-fp-atomics",
    "-Wno-unused-result",
]

HIP_SOURCES = sorted(glob.glob(os.path.join(HERE, "csrc", "kernels", "*.hip")))
HIP_HEADERS = sorted(glob.glob(os.path.join(HERE, "csrc", "kernels", "*.h"))) + [
    os.path.join(HERE, "csrc", "common.h")
]


def _hip_object(src):
    return os.path.join(HIP_OBJ_DIR, os.path.basename(src).replace(".hip", ".o"))


def compile_hip_objects(jobs=None):
    """hipcc-compile the kernel library; returns the object paths."""
    os.makedirs(HIP_OBJ_DIR, exist_ok=True)
    hdr_mtime = max(os.path.getmtime(h) for h in HIP_HEADERS)

    def build_one(src):
        obj = _hip_object(src)
        if os.path.exists(obj) and os.path.getmtime(obj) >= max(os.path.getmtime(src), hdr_mtime):
            return obj
        cmd = [os.path.join(ROCM, "bin", "hipcc"), *HIP_FLAGS, "-I", os.path.join(HERE, "csrc"),
               "-c", src, "-o", obj]
        print("[hipcc]", os.path.basename(src), flush=True)
        r = subprocess.run(cmd, capture_output=True, text=True)
        if r.returncode != 0:
            sys.stderr.write(r.stdout + r.stderr)
            raise RuntimeError(f"hipcc failed for {src}")
        return obj

    jobs = jobs or min(8, max(1, os.cpu_count() or 1))
    with ThreadPoolExecutor(jobs) as ex:
        return list(ex.map(build_one, HIP_SOURCES))


class BuildWithHip(BuildExtension):
    def build_extensions(self):
        objs = compile_hip_objects()
        for ext in self.extensions:
            ext.extra_objects = list(objs)
        super().build_extensions()


cpp_sources = ["csrc/bindings.cpp"]
for sub in ("proto", "ir", "runtime", "comm"):
    cpp_sources += sorted(os.path.relpath(p, HERE) for p in glob.glob(os.path.join(HERE, "csrc", sub, "*.cpp")))

torch_lib = os.path.join(os.path.dirname(torch.__file__), "lib")

ext = CppExtension(
    name="tensorframes_amd._C",
    sources=cpp_sources,
    include_dirs=[os.path.join(HERE, "csrc"), os.path.join(ROCM, "include")],
    define_macros=[("__HIP_PLATFORM_AMD__", "1"), ("USE_ROCM", "1")],
    library_dirs=[os.path.join(ROCM, "lib"), torch_lib],
    libraries=["amdhip64", "hiprtc", "c10_hip", "torch_hip", "rocprofiler-sdk-roctx", "rccl"],
    extra_compile_args=["-O3", "-std=c++17", "-g0", "-Wno-unused-function", "-Wno-sign-compare"],
    extra_link_args=[f"-Wl,-rpath,{os.path.join(ROCM, 'lib')}"],
)

setup(
    name="tensorframes_amd",
    version="0.1.0",
    description="MI355X-native DataFrame tensor engine with the TensorFrames API",
    packages=find_packages(include=["tensorframes_amd", "tensorframes_amd.*"]),
    ext_modules=[ext],
    cmdclass={"build_ext": BuildWithHip.with_options(use_ninja=True)},
)
