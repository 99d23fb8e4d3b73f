#!/bin/bash
# Build the GEMM/conv kernel lab (scripts/gemm_lab.cpp) against the in-tree
# kernel objects (python setup.py build_ext --inplace builds build/hip/*.o).
set -euo pipefail
cd "$(dirname "$0")/.."
mkdir -p build/lab
HIPCC=/opt/rocm/bin/hipcc
$HIPCC -O2 -std=c++17 --offload-arch=gfx950 -I csrc -x hip -c scripts/gemm_lab.cpp -o build/lab/gemm_lab.o
g++ -O2 -std=c++17 -I csrc -c scripts/gemm_lab_stubs.cpp -o build/lab/stubs.o
# every kernel object (the conv entry point dispatches to the direct conv
# kernels, the reductions to the groupby radix helpers); GEMM_O swaps in an
# alternative build of gemm.hip (e.g. other compiler flags)
GEMM_O=${GEMM_O:-build/hip/gemm.o}
OBJS=$(ls build/hip/*.o | grep -v '/gemm\.o$')
$HIPCC --hip-link --offload-arch=gfx950 build/lab/gemm_lab.o build/lab/stubs.o "$GEMM_O" $OBJS \
  -o "${OUT:-build/gemm_lab}"
echo "built ${OUT:-build/gemm_lab}"
