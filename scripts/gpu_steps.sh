#!/bin/bash
# GPU check: named steps, each under its own time limit; stops at the
# first step that faults, aborts or times out (scripts/gpu_check.sh runner).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
# clocks / power / temperature every 5 s next to every number this call
# measures (gpurun_out/smi_trace.log); SMI=0 turns it off
if [ "${SMI:-1}" = 1 ]; then
  ( while true; do echo "== $(date +%T)"; rocm-smi --showclocks --showpower --showtemp --showuse 2>&1 | grep -E "GPU\[|sclk|mclk|fclk|Power|Temperature|use"; sleep 5; done ) >> gpurun_out/smi_trace.log 2>&1 &
  SMI_PID=$!
  trap 'kill $SMI_PID 2>/dev/null' EXIT
fi
run() {
  local name=$1; shift
  local secs=$1; shift
  echo "== $name ($(date +%T))"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc"
  tail -n 4 "gpurun_out/$name.log"
  if grep -qiE "memory access fault|illegal address|hipErrorIllegal|HSA_STATUS_ERROR|core dumped" "gpurun_out/$name.log"; then
    echo "GPU fault in $name: stopping"; exit 99
  fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in ${STEPS:-tests}; do
  case $s in
    pmc) run pmc 900 bash scripts/pmc_gemm.sh ;;
    engine) run engine 300 python -u -m pytest tests/test_gpu_engine.py tests/test_streaming.py tests/test_gpu_string_keys.py -x -v --timeout 120 --timeout-method thread ;;
    comm_bench) run comm_bench 300 python scripts/comm_bench.py ;;
    comm_bench2) TFA_DIST_BACKEND=gloo run comm_bench2 300 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29517 scripts/comm_bench.py ;;
    read_image) run read_image 600 python examples/read_image.py --images 2048 ;;
    incep_bf16x3) run incep_bf16x3 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 --precision bf16x3 ;;
    incep_bf16) run incep_bf16 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 --precision bf16 ;;
    f64gemm) run f64gemm 600 python scripts/gemm_bench.py --f64-only ;;
    strkeys) run strkeys 300 python -u -m pytest tests/test_gpu_string_keys.py -x -v -s --timeout 120 --timeout-method thread ;;
    comm) run comm 300 python -u -m pytest tests/test_gpu_comm.py tests/test_rccl.py tests/test_multirank_gpu.py -x -v --timeout 120 --timeout-method thread ;;
    tests) run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    newtests) run newtests 600 python -u -m pytest tests/test_plan_reuse.py tests/test_gpu_engine.py tests/test_models.py tests/test_gpu_models.py tests/test_fusion.py -x -q --timeout 120 --timeout-method thread ;;
    ab) for i in 1 2; do run ab_old_$i 300 python ab_old/scripts/gemm_bench.py --json gpurun_out/ab_old_$i.json; run ab_new_$i 300 python scripts/gemm_bench.py --json gpurun_out/ab_new_$i.json; done ;;
    incep1m) run incep1m 900 python bench/configs.py inception --rows 1000000 --steps 1 --warmup 1 ;;
    incep1m_u8) run incep1m_u8 900 python bench/configs.py inception --rows 1000000 --steps 1 --warmup 1 --input-dtype uint8 ;;
    incep_dev) run incep_dev 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 ;;
    prof_kmeans) export TMPDIR=/tmp; run prof_kmeans 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_kmeans" -o run -- python scripts/kmeans_profile.py --iters 20 ;;
    prof_reduce) export TMPDIR=/tmp; run prof_reduce 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_reduce" -o run -- python bench/configs.py reduce --steps 2 --warmup 1 ;;
    prof_bench) export TMPDIR=/tmp; run prof_bench 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_bench" -o run -- python bench.py --steps 3 --warmup 1 ;;
    prof_incep) export TMPDIR=/tmp; run prof_incep 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_incep" -o run -- python bench/configs.py inception --source device --rows 8192 --steps 1 --warmup 1 ;;
    sib) run sib 600 python -u -m pytest tests/test_sibling_fusion.py -x -q --timeout 120 --timeout-method thread ;;
    kparts) run kparts 300 python scripts/kmeans_parts.py gpurun_out/kparts_cprofile.txt ;;
    kparts_plan) TFA_PLAN_TIMING=1 run kparts_plan 300 python scripts/kmeans_parts.py ;;
    kmeans_agg) run kmeans_agg 300 python scripts/kmeans_profile.py --iters 50 --variant aggregate ;;
    kbreak) run kbreak 300 python scripts/kmeans_breakdown.py --iters 200 ;;
    kmeans) run kmeans 300 python scripts/kmeans_profile.py --iters 50 ;;
    r4_kmeans) mkdir -p gpurun_out/r4_kmeans; export TMPDIR=/tmp
      run r4_kmeans/in_graph 300 python scripts/kmeans_profile.py --iters 200 &&
      run r4_kmeans/aggregate 300 python scripts/kmeans_profile.py --iters 200 --variant aggregate &&
      run r4_kmeans/phases 300 python scripts/kmeans_phases.py --iters 300 &&
      run r4_kmeans/cprofile 300 python scripts/kmeans_profile.py --iters 50 --cprofile &&
      run r4_kmeans/rocprof 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/r4_kmeans/rocprof" -o run -- python scripts/kmeans_profile.py --iters 20 ;;
    kmeans_cprof) run kmeans_cprof 300 python scripts/kmeans_profile.py --iters 20 --cprofile ;;
    refperf) run refperf 600 python bench/configs.py refperf ;;
    cfg_add) run cfg_add 600 python bench/configs.py add ;;
    cfg_plumbing) run cfg_plumbing 300 python bench/configs.py plumbing ;;
    cfg_reduce) run cfg_reduce 900 python bench/configs.py reduce ;;
    bench) run bench 900 python bench.py --steps 5 --warmup 2 ;;
    smi) run smi_$(date +%H%M%S) 60 rocm-smi --showclocks --showpower --showtemp --showuse ;;
    rehearse2) TFA_DIST_BACKEND=gloo run rehearse2 600 python -m torch.distributed.run --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29513 scripts/multirank_rehearsal.py ;;
    incep_sweep2) for b in 2048 4096 8192; do run incep_b$b 600 python bench/configs.py inception --source device --rows 16384 --batch $b --steps 2 --warmup 1; done ;;
    incep_host_sweep2) for c in 1024 2048; do run incep_host_c$c 900 python bench/configs.py inception --rows 65536 --batch 4096 --chunk-images $c --steps 1 --warmup 1; done ;;
    incep_sweep) for b in 256 512 1024 2048; do run incep_b$b 600 python bench/configs.py inception --source device --rows 8192 --batch $b --steps 2 --warmup 1; done ;;
    incep_host_sweep) for c in 256 1024; do run incep_host_c$c 900 python bench/configs.py inception --rows 65536 --batch 2048 --chunk-images $c --steps 1 --warmup 1; done ;;
    incep) run incep 900 python bench/configs.py inception --source device --rows ${INC_ROWS:-8192} --batch ${INC_BATCH:-512} --steps 1 --warmup 1 ;;
    wino) run wino_tests 400 python -u -m pytest tests/test_gpu_wino.py -x -v --timeout 200 --timeout-method thread &&
      run layers_wino 700 python scripts/conv_layers.py --json gpurun_out/layers_wino.json &&
      TFA_CONV_ALGO=direct run layers_direct 700 python scripts/conv_layers.py --json gpurun_out/layers_direct.json ;;
    wino_pmc) export TMPDIR=/tmp
      for spec in ${WINO_PMC:-4:0 4:1 8:1 2:1}; do set -- ${spec/:/ }
        for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE" \
                    "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE" \
                    "TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum GRBM_GUI_ACTIVE"; do
          tag=l$1_v$2_$(echo $pass | cut -c1-6)
          TFA_WINO_TILE=$2 run pmc_$tag 120 rocprofv3 --pmc $pass --output-format csv -d "$PWD/gpurun_out/wino_pmc/$tag" -o run -- python scripts/conv_layers.py --only $1 --iters 2 || exit 1
        done
      done ;;
    wtest) run wino_tests 400 python -u -m pytest tests/test_gpu_wino.py -x -v --timeout 200 --timeout-method thread ;;
    layers_v1) run layers_wino_v1 700 python scripts/conv_layers.py --json gpurun_out/layers_wino_v1.json ;;
    wdbg) for d in ${WDBG:-0 1 2 3 4}; do TFA_WINO_DEBUG=$d run wdbg_l${WL:-4}_d$d 120 python scripts/conv_layers.py --only ${WL:-4} --iters 5 || exit 1; grep -h TF gpurun_out/wdbg_l${WL:-4}_d$d.log | tail -1; done ;;
    wsweep) run wsweep 300 python scripts/wino_sweep.py ;;
    wsweep3) TFA_WINO_TILE=3 run wsweep3 300 python scripts/wino_sweep.py ;;
    layers_v2) TFA_WINO_TILE=2 run layers_wino_v2 700 python scripts/conv_layers.py --json gpurun_out/layers_wino_v2.json ;;
    layers_bn32) TFA_WINO_BN=32 run layers_bn32 700 python scripts/conv_layers.py --json gpurun_out/layers_bn32.json ;;
    layers_v0) TFA_WINO_TILE=0 run layers_wino_v0 700 python scripts/conv_layers.py --json gpurun_out/layers_wino_v0.json ;;
    kmeans_cfg) run kmeans_cfg 300 python bench/configs.py kmeans ;;
    gemm_bench) run gemm_bench 600 python scripts/gemm_bench.py --json gpurun_out/gemm_bench.json ;;
    tune_log) TFA_GEMM_TUNE_LOG=1 run tune_log 600 python bench/configs.py inception --source device --rows 4096 --steps 1 --warmup 1 ;;
    incep_s3) TFA_CONCURRENT_LARGE_STREAMS=3 run incep_s3 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 ;;
    incep_serial) TFA_CONCURRENT_LARGE=0 run incep_serial 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 ;;
    bench_ab) for i in 1 2; do
        run bench_s2_$i 600 python bench.py --steps 5 --warmup 2 &&
        TFA_PIPE_COMPUTE_STREAMS=1 run bench_s1_$i 600 python bench.py --steps 5 --warmup 2 || exit 1; done ;;
    steptest) run steptest 300 python -u -m pytest tests/test_gpu_step_timing.py tests/test_gpu_overlap.py -x -v --timeout 120 --timeout-method thread ;;
    slim) run read_image4k_slim 400 python examples/read_image.py --images 4096 --prep slim ;;
    # ---- round 6: the executed plan (per-step device time) and one timed window's kernel trace
    layers_exec)
      run layers_exec_incep 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 --step-profile gpurun_out/layers_exec_incep.json &&
      run layers_exec_vgg 600 python examples/read_image.py --images 4096 --step-profile gpurun_out/layers_exec_vgg.json ;;
    trace_incep) export TMPDIR=/tmp
      run trace_incep 900 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$PWD/gpurun_out/trace_incep" -o run -- python bench/configs.py inception --source device --rows 16384 --steps 1 --warmup 1 &&
      run trace_incep_window 120 python scripts/trace_window.py gpurun_out/trace_incep --out gpurun_out/trace_incep_step.md --title "Inception-v3, 16384 device-resident images: one timed step" ;;
    trace_vgg) export TMPDIR=/tmp
      run trace_vgg 600 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$PWD/gpurun_out/trace_vgg" -o run -- python examples/read_image.py --images 4096 &&
      run trace_vgg_window 120 python scripts/trace_window.py gpurun_out/trace_vgg --out gpurun_out/trace_vgg_step.md --title "VGG-16 JPEG scoring (read_image), 4096 images: the steady-state pass" ;;
    # ---- presets (the one-off round-4/5 step lists, folded in)
    final) STEPS=smoke bash scripts/gpu_check.sh && run tests 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
      run bench 900 python bench.py --steps 5 --warmup 2 &&
      run incep_dev 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 ;;
    prec) run prec 300 python -u -m pytest tests/test_gpu_precision.py tests/test_gpu_g2.py -x -q --timeout 300 --timeout-method thread ;;
    tile_ab) run tile_ab 900 bash scripts/tile_ab.sh ;;                    # SHAPES=<file> TILES="auto 16 28 ..."
    ab2)  # forced-tile A/B of single shapes: AB="name|tiles|gemm_one args;..."
      IFS=';' read -ra items <<< "${AB:-}"
      for it in "${items[@]}"; do IFS='|' read -r nm tiles args <<< "$it"
        for t in $tiles; do TFA_GEMM_TILE=$t run ab_${nm}_t$t 120 python scripts/gemm_one.py $args --iters 10 || exit 1; done
      done ;;
    g2_ab)  # g2 core correctness, then forced-tile A/B: TILES / HEAD_TILES / CONV_TILES
      run g2_tests 400 python -u -m pytest tests/test_gpu_g2.py tests/test_gpu_precision.py -x -q --timeout 300 --timeout-method thread || exit 1
      for t in ${TILES:-21 22 23 24}; do
        TFA_GEMM_TILE=$t run ab_4096_t$t 120 python scripts/gemm_one.py gemm 4096 4096 4096 --iters 30 &&
        TFA_GEMM_TILE=$t run ab_4096tb_t$t 120 python scripts/gemm_one.py gemm 4096 4096 4096 --iters 30 --tb &&
        TFA_GEMM_TILE=$t run ab_8192_t$t 120 python scripts/gemm_one.py gemm 8192 8192 8192 --iters 10 || exit 1
      done
      for t in ${HEAD_TILES:-13 22 23 24 25}; do TFA_GEMM_TILE=$t run ab_head_t$t 120 python scripts/gemm_one.py gemm 2500000 512 512 --iters 20 || exit 1; done
      for t in ${CONV_TILES:-16 23 24 25 26}; do TFA_GEMM_TILE=$t run ab_conv4a_t$t 120 python scripts/gemm_one.py conv 2048 54 54 80 3 3 192 1 VALID --iters 10 || exit 1; done ;;
    lab_g2)  # the g2 GEMM lab kernel (scripts/g2_lab.hip) on G2_SHAPES; counters with PMC=1
      export TMPDIR=/tmp
      hipcc -O3 --offload-arch=gfx950 -std=c++17 scripts/g2_lab.hip -o /tmp/g2_lab || exit 3
      for shape in ${G2_SHAPES:-"4096 4096 4096" "8192 8192 8192" "2560000 512 512"}; do
        run lab_g2_${shape// /x} 120 /tmp/g2_lab $shape || exit 1; done
      if [ -n "${PMC:-}" ]; then
        PA="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE"
        PB="SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAVES SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"
        timeout -s KILL 90 rocprofv3 --pmc $PA --output-format csv -d "$PWD/gpurun_out/lab_pmc/a" -o run -- /tmp/g2_lab 4096 4096 4096 one > gpurun_out/lab_pmc_a.log 2>&1 &&
        timeout -s KILL 90 rocprofv3 --pmc $PB --output-format csv -d "$PWD/gpurun_out/lab_pmc/b" -o run -- /tmp/g2_lab 4096 4096 4096 one > gpurun_out/lab_pmc_b.log 2>&1 || exit 1
      fi ;;
    tile_table_vgg) run tile_table_vgg 600 python scripts/tile_table.py --add-read-image --out gpurun_out/gfx950.json ;;
    tile_table) run tile_table 1000 python scripts/tile_table.py --out gpurun_out/gfx950.json ;;
    layers_time) run layers_time 700 python scripts/conv_layers.py --json gpurun_out/layers.json ;;
    layers_pmc) run layers_pmc 1150 python scripts/layers_pmc.py --layers scripts/data/inception_layers.json --out gpurun_out/layers_pmc --first ${FIRST:-0} --last ${LAST:-21} ;;
    img) run img_tests 300 python -u -m pytest tests/test_gpu_image_prep.py tests/test_jpeg_native.py tests/test_gpu_string_keys.py -x -v -s --timeout 200 --timeout-method thread &&
      run read_image4k 400 python examples/read_image.py --images 4096 &&
      TFA_PRECISION=bf16x3 run read_image4k_bf16x3 400 python examples/read_image.py --images 4096 ;;
    decode_bench) run decode_bench 300 python scripts/decode_bench.py --images 1024 ;;
    pool) run pool 400 python -u -m pytest tests/test_gpu_pool_accounting.py tests/test_multirank_gpu.py tests/test_gpu_engine.py -x -v --timeout 200 --timeout-method thread ;;
    poolb)
      TFA_POOL_GENERIC=1 run pool_generic 300 python scripts/pool_bench.py &&
      TFA_POOL_XCD=0 run pool_3x3 300 python scripts/pool_bench.py &&
      run pool_3x3_xcd 300 python scripts/pool_bench.py ;;
    stemx) run stem_tests 300 python -u -m pytest tests/test_gpu_conv_direct.py tests/test_gpu_conv_smallc.py -x -q --timeout 120 --timeout-method thread &&
      TFA_SMALLC_GENERIC=1 run stem_gen_l0 300 python scripts/conv_layers.py --only 0 &&
      run stem_fast_l0 300 python scripts/conv_layers.py --only 0 ;;
    f45) run f45_tests 400 python -u -m pytest tests/test_gpu_wino.py tests/test_wino.py -x -v --timeout 200 --timeout-method thread &&
      run incep_dev_no5x5 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 --step-profile gpurun_out/layers_no5x5.json &&
      TFA_WINO_5X5=1 run incep_dev_f45 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 --step-profile gpurun_out/layers_f45.json &&
      run incep_dev_no5x5_2 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 &&
      TFA_WINO_5X5=1 run incep_dev_f45_2 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 ;;
    vgg_serial) TFA_CONCURRENT_LARGE=0 run vgg_serial 400 python examples/read_image.py --images 4096 --step-profile gpurun_out/vgg_serial.json ;;
    prio_ab) for i in 1 2; do for pr in 0 1; do
        TFA_WINO_PRIO=$pr run prio${pr}_l4_$i 200 python scripts/conv_layers.py --only 4 --iters 20 &&
        TFA_WINO_PRIO=$pr run prio${pr}_l2_$i 200 python scripts/conv_layers.py --only 2 --iters 20 &&
        TFA_WINO_PRIO=$pr run prio${pr}_l9_$i 200 python scripts/conv_layers.py --only 9 --iters 20 || exit 1; done; done
      grep -h '"layer"' gpurun_out/prio*_l*.log | cut -c1-200 ;;
    poolconv) run poolconv_tests 300 python -u -m pytest tests/test_gpu_pool_conv.py tests/test_pool_conv_plan.py tests/test_gpu_conv_smallc.py -x -v --timeout 120 --timeout-method thread &&
      TFA_POOL_CONV_FUSION=0 TFA_CONCURRENT_LARGE=0 run incep_serial_nopc 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 --step-profile gpurun_out/layers_nopc.json &&
      TFA_POOL_CONV_FUSION=1 TFA_CONCURRENT_LARGE=0 run incep_serial_pc 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 --step-profile gpurun_out/layers_pc.json &&
      TFA_POOL_CONV_FUSION=1 TFA_POOLCONV_WS=0 TFA_CONCURRENT_LARGE=0 run incep_serial_pc_nows 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 --step-profile gpurun_out/layers_pc_nows.json &&
      TFA_POOL_CONV_FUSION=0 run incep_dev_nopc 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 &&
      TFA_POOL_CONV_FUSION=1 run incep_dev_pc 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 ;;
    smallc_tr) run stem_tests 300 python -u -m pytest tests/test_gpu_conv_smallc.py tests/test_gpu_conv_direct.py -x -q --timeout 120 --timeout-method thread &&
      for i in 1 2; do for tr in 0 1; do
        TFA_SMALLC_TR=$tr run tr${tr}_l0_$i 200 python scripts/conv_layers.py --only 0 --iters 20 || exit 1; done; done &&
      TFA_SMALLC_TR=0 TFA_CONCURRENT_LARGE=0 run vgg_tr0 400 python examples/read_image.py --images 4096 --step-profile gpurun_out/vgg_tr0.json &&
      TFA_CONCURRENT_LARGE=0 run vgg_tr1 400 python examples/read_image.py --images 4096 --step-profile gpurun_out/vgg_tr1.json ;;
    bench2r) TFA_DIST_BACKEND=gloo TFA_BENCH_REHEARSAL=1 run bench_2ranks_1gpu 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 ;;
    layers_vgg) run layers_vgg 600 python scripts/conv_layers.py --model vgg16 --json gpurun_out/layers_vgg.json ;;
    add_chunks) for c in 16 8 4 32; do TFA_MIN_PIPELINE_CHUNKS=$c run cfg_add_c$c 300 python bench/configs.py add --steps 10 --warmup 3 || exit 1; done
      grep -ho '"value": [0-9.]*' gpurun_out/cfg_add_c*.log ;;
    smallc_ws) TFA_SMALLC_WS=1 run stem_tests_ws 300 python -u -m pytest tests/test_gpu_conv_smallc.py -x -q --timeout 120 --timeout-method thread &&
      for i in 1 2; do for w in 0 1; do
        TFA_SMALLC_WS=$w run ws${w}_l0_$i 200 python scripts/conv_layers.py --only 0 --iters 20 || exit 1; done; done &&
      TFA_CONCURRENT_LARGE=0 run vgg_ws0 400 python examples/read_image.py --images 4096 --step-profile gpurun_out/vgg_ws0.json &&
      TFA_SMALLC_WS=1 TFA_CONCURRENT_LARGE=0 run vgg_ws1 400 python examples/read_image.py --images 4096 --step-profile gpurun_out/vgg_ws1.json ;;
    optin_tests) TFA_WINO_5X5=1 run tests_wino5x5 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread &&
      TFA_POOL_CONV_FUSION=0 run tests_nopoolconv 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread ;;
    incep_sweep3) for b in 1024 2048 4096; do run incep3_b$b 600 python bench/configs.py inception --source device --rows 16384 --batch $b --steps 2 --warmup 1 || exit 1; done
      for c in 512 1024 2048; do run incep3_host_c$c 900 python bench/configs.py inception --rows 65536 --chunk-images $c --steps 1 --warmup 1 || exit 1; done ;;
    incep_sweep4) for b in 4096 2048; do run incep4_b$b 600 python bench/configs.py inception --source device --rows 16384 --batch $b --steps 2 --warmup 1 || exit 1; done
      run incep4_1m_c2048 900 python bench/configs.py inception --rows 1000000 --chunk-images 2048 --steps 1 --warmup 1 &&
      run incep4_1m_c1024 900 python bench/configs.py inception --rows 1000000 --chunk-images 1024 --steps 1 --warmup 1 ;;
    stem64) run stem_tests 300 python -u -m pytest tests/test_gpu_conv_smallc.py tests/test_gpu_conv_direct.py -x -q --timeout 120 --timeout-method thread &&
      run stem64_l0_b4096 200 python scripts/conv_layers.py --only 0 --batch 4096 --iters 10 &&
      run stem64_incep_dev 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 &&
      run stem64_read_image 400 python examples/read_image.py --images 4096 &&
      TFA_MAP_ROWS_BATCH=512 run stem64_read_image_b512 400 python examples/read_image.py --images 4096 ;;
    incep_sweep5) run incep5_b8192 600 python bench/configs.py inception --source device --rows 16384 --batch 8192 --steps 2 --warmup 1 &&
      run incep5_b4096 600 python bench/configs.py inception --source device --rows 16384 --batch 4096 --steps 2 --warmup 1 &&
      run incep5_1m_b4096_c4096 900 python bench/configs.py inception --rows 1000000 --batch 4096 --chunk-images 4096 --steps 1 --warmup 1 &&
      run incep5_1m_b4096_c2048 900 python bench/configs.py inception --rows 1000000 --batch 4096 --chunk-images 2048 --steps 1 --warmup 1 ;;
    img_batch) for b in 128 192 256 384; do TFA_MAP_ROWS_BATCH=$b run img_b$b 400 python examples/read_image.py --images 4096 || exit 1; done
      grep -h steady gpurun_out/img_b*.log ;;
    trace_bench) export TMPDIR=/tmp
      run trace_bench 900 rocprofv3 --kernel-trace --marker-trace --output-format csv -d "$PWD/gpurun_out/trace_bench" -o run -- python bench.py --steps 3 --warmup 2 &&
      run trace_bench_window 120 python scripts/trace_window.py gpurun_out/trace_bench --out gpurun_out/trace_bench_step.md --title "Headline bench.py (config 3, host-resident), 3 timed steps" ;;
    groupby) run groupby 300 python scripts/groupby_profile.py ;;
    vggstem) run stem_tests 300 python -u -m pytest tests/test_gpu_conv_direct.py tests/test_gpu_conv_smallc.py -x -q --timeout 120 --timeout-method thread &&
      TFA_SMALLC_GENERIC=1 run vgg_stem_generic 400 python examples/read_image.py --images 4096 --step-profile gpurun_out/vgg_stem_generic.json &&
      run vgg_stem_padfast 400 python examples/read_image.py --images 4096 --step-profile gpurun_out/vgg_stem_padfast.json ;;
    headab) for i in 1 2; do
        run head_default_$i 600 python bench.py --steps 3 --warmup 2 &&
        TFA_GEMM_DEFAULTS=scripts/data/gfx950_t19.json run head_t19_$i 600 python bench.py --steps 3 --warmup 2 || exit 1; done ;;
    poolk) run poolk_tests 300 python -u -m pytest tests/test_gpu_pool_fusion.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread &&
      TFA_POOL_GENERIC=1 run incep_dev_poolgen 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 &&
      run incep_dev_pool3 900 python bench/configs.py inception --source device --rows 16384 --steps 2 --warmup 1 &&
      export TMPDIR=/tmp && run prof_incep 900 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/gpurun_out/prof_incep" -o run -- python bench/configs.py inception --source device --rows 8192 --steps 1 --warmup 1 ;;
  esac
done
echo "all steps done"
