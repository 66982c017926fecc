#!/bin/bash
# tools/r06_final_a.sh — round 6's evidence, part A (one gpurun call): GPU test suite, smoke,
# PMC profiles of PROF_CFGS (tools/round_profile.sh).  Part B: more PROF_CFGS; part C:
# tools/round_bench.sh.  Collected on the build host with tools/collect_round.py.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
if [ -n "${WITH_TESTS:-}" ]; then
  timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
      > gpurun_out/gpu_tests_final.log 2>&1 || { echo "gpu tests failed"; tail -30 gpurun_out/gpu_tests_final.log; exit 1; }
  tail -1 gpurun_out/gpu_tests_final.log
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; exit 1; }
  tail -1 gpurun_out/smoke.log
fi
bash tools/round_profile.sh
