#!/bin/bash
# tools/final_profile.sh — the round's evidence for the library in the tree, on the
# gpurun box: PMC passes of the timed c4 megakernel (separate rocprofv3 passes) and
# their summary (traffic.json, read by bench.py's roofline), a kernel-trace --stats
# run of bench.py, and the bench lines of c4 (with the CPU baseline), c2, c3, c5.
# Every step under its own time limit; the first failure ends the script.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/final
mkdir -p $O
B="python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline"
for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_HIT_sum TCC_MISS_sum:l2" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE:sq"; do
  ctrs=${pass%%:*}; name=${pass##*:}
  echo "== pmc $name"
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc_$name -o run --output-format csv -- $B > $O/pmc_$name.log 2>&1
done
python3 tools/pmc_traffic.py $O $O/summary 250000000 c4
echo "== kernel trace"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
    python3 bench.py --config c4 --steps 5 --warmup 1 --no-cpu-baseline > $O/prof.log 2>&1
echo "== bench c4"
timeout -k 10 400 python3 bench.py > $O/bench_c4.log 2>&1
for c in c2 c3 c5; do
  echo "== bench $c"
  timeout -k 10 300 python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $O/bench_$c.log 2>&1
done
echo done
