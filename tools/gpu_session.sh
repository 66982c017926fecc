#!/bin/bash
# tools/gpu_session.sh STEP... — runs named GPU steps on the gpurun box, each under
# its own time limit; logs go to gpurun_out/<step>.log.  A step that exits 0 or 1
# (tests failed / assertion) lets the next step run; any other status (fault,
# abort, segfault, timeout) ends the session there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
run() {
  local name=$1 t=$2; shift 2
  echo "== $name: $*" >> gpurun_out/steps.txt
  local t0=$(date +%s)
  timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 ))s" | tee -a gpurun_out/steps.txt
  tail -3 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
}
for step in "$@"; do
  case $step in
    build)  run build 600 python -c "import __graft_entry__ as g; g.build()" ;;
    smoke)  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    tests)  run tests 1200 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread ;;
    testsk) run tests 1200 python -m pytest tests -m gpu -q -s ;;
    bench_small) run bench_small 600 python bench.py --spp 64 --steps 2 --warmup 1 --no-cpu-baseline ;;
    bench)  run bench 900 python bench.py ;;
    prof)   export TMPDIR=/tmp
            run prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --config ${BENCH_CFG:-c4} --steps 5 --warmup 1 --no-cpu-baseline ;;
    counters) export TMPDIR=/tmp; run counters 120 rocprofv3 -L ;;
    pmc_fetch) export TMPDIR=/tmp
            run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
    pmc_write) export TMPDIR=/tmp
            run pmc_write 900 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
    pmc_l2) export TMPDIR=/tmp
            run pmc_l2 900 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
    pmc_sq) export TMPDIR=/tmp
            run pmc_sq 900 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline ;;
    stages) run stages 600 python3 tools/stage_profile.py final ;;
    stages_cornell) run stages_cornell 600 python3 tools/stage_profile.py cornell_box ;;
    dist2)  run dist2 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --spp 64 --steps 2 --warmup 1 --ppm gpurun_out/dist2.ppm ;;
    one_ppm) run one_ppm 600 python3 bench.py --spp 64 --steps 1 --warmup 0 --no-cpu-baseline --ppm gpurun_out/one.ppm ;;
    pmc)    export TMPDIR=/tmp   # BENCH_CFG=c4|c5|c2|c3 (default c4)
            B="python3 bench.py --config ${BENCH_CFG:-c4} --steps 1 --warmup 0 --no-cpu-baseline"
            run pmc_fetch 300 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/pmc_fetch -o run --output-format csv -- $B
            run pmc_write 300 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/pmc_write -o run --output-format csv -- $B
            run pmc_l2 300 timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum -d gpurun_out/pmc_l2 -o run --output-format csv -- $B
            run pmc_sq 300 timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE -d gpurun_out/pmc_sq -o run --output-format csv -- $B ;;
    pmc_deep) export TMPDIR=/tmp
            B="python3 bench.py --spp ${PMC_SPP:-128} --steps 1 --warmup 0 --no-cpu-baseline"
            run pmc_d2 600 rocprofv3 --pmc TA_TA_BUSY GRBM_GUI_ACTIVE -d gpurun_out/pmc_d2 -o run --output-format csv -- $B
            run pmc_d3 600 rocprofv3 --pmc TD_TD_BUSY -d gpurun_out/pmc_d3 -o run --output-format csv -- $B
            run pmc_d4 600 rocprofv3 --pmc TA_FLAT_READ_WAVEFRONTS -d gpurun_out/pmc_d4 -o run --output-format csv -- $B
            run pmc_d5 600 rocprofv3 --pmc TCP_TOTAL_CACHE_ACCESSES -d gpurun_out/pmc_d5 -o run --output-format csv -- $B
            run pmc_d6 600 rocprofv3 --pmc TCP_CACHE_MISS -d gpurun_out/pmc_d6 -o run --output-format csv -- $B
            run pmc_d7 600 rocprofv3 --pmc TCP_PENDING_STALL_CYCLES -d gpurun_out/pmc_d7 -o run --output-format csv -- $B
            run pmc_d8 600 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_FLAT SQ_WAIT_ANY SQ_WAIT_INST_ANY -d gpurun_out/pmc_d8 -o run --output-format csv -- $B
            run pmc_d9 600 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_FLAT SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_SMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU -d gpurun_out/pmc_d9 -o run --output-format csv -- $B
            run pmc_d10 600 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_d10 -o run --output-format csv -- $B
            python3 tools/pmc_deep.py gpurun_out > gpurun_out/pmc_deep.txt ;;
    pmc_lanes) export TMPDIR=/tmp
            B="python3 bench.py --spp ${PMC_SPP:-128} --steps 1 --warmup 0 --no-cpu-baseline"
            run pmc_l1 600 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc_l1 -o run --output-format csv -- $B ;;
    dist2n) run dist2n 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 --dist-backend gloo --spp 64 --steps 2 --warmup 1 --ppm gpurun_out/dist2n.ppm ;;
    c5one)  run c5one 600 python3 bench.py --config c5 --steps 2 --warmup 1 --no-cpu-baseline --ppm gpurun_out/c5one.ppm ;;
    lanes)  export TMPDIR=/tmp   # VALU lane utilisation of the timed kernel, per config (LANES_CFGS)
            for c in ${LANES_CFGS:-c4 c2 c3}; do
              run lanes_$c 300 timeout -s KILL 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/lanes_$c -o run --output-format csv -- python3 bench.py --config $c --steps 1 --warmup 0 --no-cpu-baseline
            done
            run lanes_sum 60 python3 tools/lanes_summary.py gpurun_out gpurun_out/lanes.json ;;
    dist2s) run dist2s 600 python3 bench.py --gpus 2 --dist-backend gloo --spp 64 --steps 2 --warmup 1 --no-cpu-baseline --dump gpurun_out/dist2s.npy ;;
    probe)  run probe 600 python3 tools/scaling_probe.py --out gpurun_out/scaling_probe.json ;;
    c5)     run c5 600 python3 bench.py --config c5 --steps 3 --warmup 1 --no-cpu-baseline ;;
    pmcsum) run pmcsum 60 python3 tools/pmc_traffic.py gpurun_out gpurun_out/profile_summary 250000000 c4 ;;
    ab)     run ab 1200 python3 tools/ab.py $AB_LIBS --rounds ${AB_ROUNDS:-2} ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
