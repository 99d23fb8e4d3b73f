#!/bin/bash
# GPU box: config 5 (Inception-v3 over a host-resident image column) at BASELINE scale.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg5
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
ROWS=${ROWS:-1000000}
step() { local name=$1; shift; echo "== $name $(date +%T)"; timeout -k 10 "$@" > gpurun_out/cfg5/$name.log 2>&1; local rc=$?; grep '{' gpurun_out/cfg5/$name.log; [ $rc -eq 0 ] || { echo "$name rc=$rc"; tail -25 gpurun_out/cfg5/$name.log; exit 1; }; }
step small_f32 300 python bench/configs.py inception --rows 4096 --batch 1024 --steps 1 --warmup 1
step small_u8 300 python bench/configs.py inception --rows 4096 --batch 1024 --steps 1 --warmup 1 --input-dtype uint8
step prof_f32 400 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d gpurun_out/cfg5/prof_f32 -o run -- python bench/configs.py inception --rows 16384 --batch 2048 --steps 1 --warmup 1
step full_f32 600 python bench/configs.py inception --rows $ROWS --batch 2048 --steps 1 --warmup 1
step full_u8 600 python bench/configs.py inception --rows $ROWS --batch 2048 --steps 1 --warmup 1 --input-dtype uint8
step dev_f32 300 python bench/configs.py inception --source device --rows 16384 --batch 512 --steps 2 --warmup 1
