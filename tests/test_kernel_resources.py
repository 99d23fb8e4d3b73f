"""Register/scratch budget of the MFMA GEMM kernels (compile-time check, no GPU).

A GEMM whose accumulator array is indexed with a runtime value anywhere (e.g.
an epilogue loop the unroller gives up on) keeps the whole array in scratch and
stores every accumulator once per k tile: the f64 GEMM fell from 59 to 25 TF
that way (profiles/r2_gemm_noscratch/). hipcc's resource-usage remarks show it
as ScratchSize > 0, so the kernels are compiled for gfx950 here and checked.
gemm.hip itself takes minutes to compile and is covered by the same pattern
(static_for over the accumulator tiles); the two smaller files are checked.
"""
import os
import re
import shutil
import subprocess

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = os.path.join(os.environ.get("ROCM_PATH", "/opt/rocm"), "bin", "hipcc")


def _resources(src, tmp_path):
    out = tmp_path / "k.o"
    cmd = [HIPCC, "-O3", "-std=c++17", "--offload-arch=gfx950", "-fPIC", "-ffp-contract=fast",
           "-munsafe-fp-atomics", "-I", os.path.join(REPO, "csrc"), "--cuda-device-only", "-c",
           "-Rpass-analysis=kernel-resource-usage", os.path.join(REPO, "csrc", "kernels", src), "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    kernels, cur = {}, None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\S+)", line)
        if m:
            cur = m.group(1)
            kernels[cur] = {}
            continue
        for key in ("ScratchSize [bytes/lane]", "VGPRs Spill"):
            m = re.search(re.escape(key) + r": (\d+)", line)
            if m and cur:
                kernels[cur][key] = int(m.group(1))
    return kernels


@pytest.mark.skipif(not shutil.which(HIPCC) and not os.path.exists(HIPCC), reason="hipcc not available")
@pytest.mark.parametrize("src,prefix", [("gemm_f64.hip", "gemm_f64_mfma"), ("gemm_bf16.hip", "gemm_bf16_tile")])
def test_gemm_kernels_use_no_scratch(src, prefix, tmp_path):
    kernels = _resources(src, tmp_path)
    gemms = {k: v for k, v in kernels.items() if prefix in k}
    assert gemms, f"no {prefix} kernels found in {src}"
    bad = {k: v for k, v in gemms.items() if v.get("ScratchSize [bytes/lane]", 0) or v.get("VGPRs Spill", 0)}
    assert not bad, f"GEMM kernels spilling to scratch: {bad}"
