#!/bin/bash
# tools/ab_session.sh — one A/B session on the gpurun box (edit the variants): the GPU
# parity tests with the in-tree library, then tools/ab.py over libraries / environment
# settings given in AB_ARGS (c4; @--config+c3 for c3, @--share-of+8 for a c5 rank share).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
TAG=${1:-ab}
timeout -k 10 600 python3 -u -m pytest ${TESTS:-tests} -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
if [ -n "${TEST_LIB:-}" ]; then   # the parity tests again with a variant library
  RTNW_LIB=$TEST_LIB timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 \
      --timeout-method thread > gpurun_out/${TAG}_tests_lib.log 2>&1 || { echo "variant tests failed"; tail -30 gpurun_out/${TAG}_tests_lib.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests_lib.log
fi
# AB_ARGS: tools/ab.py arguments (libraries, @config suffixes, --rounds)
timeout -k 10 900 python3 tools/ab.py ${AB_ARGS} > gpurun_out/${TAG}.log 2>&1
echo "ab rc=$?"; grep SUMMARY gpurun_out/${TAG}.log
