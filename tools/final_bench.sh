#!/bin/bash
# tools/final_bench.sh — after tools/final_profile.sh and the committed summary: a
# kernel-trace --stats run of bench.py and the bench lines of c4 (with the CPU
# baseline), c2, c3, c5, each under its own time limit.  Output: gpurun_out/final/.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
O=gpurun_out/final
mkdir -p $O
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
