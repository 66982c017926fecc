#!/bin/bash
# tools/sky_session.sh — open-sky-last ordering on the gpurun box: parity tests with the
# in-tree library, the sky split each workload gets, the launch drain with and without
# it (tools/wave_log.py), and an interleaved A/B against variants/cur (c4, c5 share of 8).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/sky
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
N=peter-shirley-ray-tracing-the-next-week_amd/librt_hip.so
C=variants/cur/librt_hip.so
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread \
    > gpurun_out/sky/tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/sky/tests.log; exit 1; }
tail -2 gpurun_out/sky/tests.log
for cfg in c4 c3 c2; do
  RTNW_TRACE=1 timeout -k 10 120 python3 bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline \
      > gpurun_out/sky/trace_$cfg.log 2>&1 || { echo "trace $cfg failed"; exit 1; }
  grep "open sky" gpurun_out/sky/trace_$cfg.log | tail -1
done
RTNW_TRACE=1 timeout -k 10 120 python3 bench.py --share-of 8 --steps 1 --warmup 0 \
    > gpurun_out/sky/trace_share8.log 2>&1 || { echo "trace share failed"; exit 1; }
grep "open sky" gpurun_out/sky/trace_share8.log | tail -1
for v in 0 1; do
  RTNW_SKY_LAST=$v timeout -k 10 180 python3 tools/wave_log.py --config c4 --out gpurun_out/sky/wave_log_c4_sky$v.json \
      > gpurun_out/sky/wave_log_c4_sky$v.log 2>&1 || { echo "wave_log $v failed"; exit 1; }
  tail -4 gpurun_out/sky/wave_log_c4_sky$v.log
done
timeout -k 10 900 python3 tools/ab.py $C "$N:RTNW_SKY_LAST=0" $N "$C@--share-of+8" "$N:RTNW_SKY_LAST=0@--share-of+8" "$N@--share-of+8" \
    --rounds 3 > gpurun_out/sky/ab.log 2>&1
echo "ab rc=$?"; grep SUMMARY gpurun_out/sky/ab.log
