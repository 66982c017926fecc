#!/bin/bash
# tools/round_all.sh — the round's whole GPU evidence for the library in the tree, in one
# gpurun call: GPU test suite, smoke, PMC profiles of every config (round_profile.sh), bench
# lines + kernel trace + wave timeline + stage profile (round_bench.sh), then an optional
# A/B (AB_ARGS: tools/ab.py arguments).  Collect on the build host with tools/collect_round.py.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    > gpurun_out/gpu_tests_final.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_final.log; exit 1; }
tail -1 gpurun_out/gpu_tests_final.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
tail -1 gpurun_out/smoke.log
PROF_CFGS="c4 c5_n8 c5 c3 c2 c5_n2 c5_n4" bash tools/round_profile.sh || exit 1
bash tools/round_bench.sh || exit 1
if [ -n "${AB_ARGS:-}" ]; then
  timeout -k 10 700 python3 tools/ab.py $AB_ARGS > gpurun_out/ab_round_all.log 2>&1
  echo "ab rc=$?"; grep SUMMARY gpurun_out/ab_round_all.log
fi
