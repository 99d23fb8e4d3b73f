#!/bin/bash
# Build the GEMM/conv kernel lab (scripts/gemm_lab.cpp) against the in-tree
# kernel objects (python setup.py build_ext --inplace builds build/hip/*.o).
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p build/lab
HIPCC=/opt/rocm/bin/hipcc
$HIPCC -O2 -std=c++17 --offload-arch=gfx950 -I csrc -x hip -c scripts/gemm_lab.cpp -o build/lab/gemm_lab.o
g++ -O2 -std=c++17 -I csrc -c scripts/gemm_lab_stubs.cpp -o build/lab/stubs.o
$HIPCC --hip-link --offload-arch=gfx950 build/lab/gemm_lab.o build/lab/stubs.o build/hip/gemm.o \
  build/hip/gemm_bf16.o build/hip/gemm_f64.o build/hip/elementwise.o build/hip/reduce.o build/hip/extra.o build/hip/image.o \
  -o build/gemm_lab
echo "built build/gemm_lab"
