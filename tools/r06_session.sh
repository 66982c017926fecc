#!/bin/bash
# tools/r06_session.sh TAG "AB_ARGS" [TESTS] — one GPU session of round 6: the GPU test suite
# (or TESTS) with the in-tree library, then tools/ab.py over AB_ARGS.  A test FAILURE (rc 1)
# still runs the A/B (timing of a wrong image is still a timing); a crash, abort or time
# limit ends the session there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/r06
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
TAG=$1
AB=${2:-}
TESTS=${3:-tests}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 900 python3 -u -m pytest $TESTS -x -q -m gpu --timeout 120 --timeout-method thread \
      > gpurun_out/r06/${TAG}_tests.log 2>&1
  rc=$?
  tail -3 gpurun_out/r06/${TAG}_tests.log
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "tests ended with rc=$rc: stopping"; exit $rc; fi
  [ $rc -eq 1 ] && grep -E "^FAILED|Error|assert" gpurun_out/r06/${TAG}_tests.log | head -20
fi
if [ -n "$AB" ]; then
  timeout -k 10 900 python3 tools/ab.py $AB > gpurun_out/r06/${TAG}_ab.log 2>&1
  echo "ab rc=$?"
  grep SUMMARY gpurun_out/r06/${TAG}_ab.log
fi
