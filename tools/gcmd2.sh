set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for v in ${VARS:-base coop coop2}; do
  RTNW_LIB=$PWD/variants/$v/librt_hip.so timeout -k 10 300 python3 tools/stage_profile.py final > gpurun_out/stage_$v.json 2> gpurun_out/stage_$v.err
  echo "stage $v rc=$?"
  RTNW_LIB=$PWD/variants/$v/librt_hip.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS -d gpurun_out/pmc_$v -o run --output-format csv -- python3 bench.py --spp 128 --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/pmc_$v.log 2>&1
  rc=$?; echo "pmc $v rc=$rc"; [ $rc -le 1 ] || exit $rc
done
timeout -k 10 900 python3 tools/ab.py variants/base/librt_hip.so variants/coop/librt_hip.so variants/coop2/librt_hip.so --rounds 3 > gpurun_out/ab2.log 2>&1
echo "ab rc=$?"; tail -4 gpurun_out/ab2.log
RTNW_LIB=$PWD/variants/coop2/librt_hip.so timeout -k 10 300 python3 bench.py --steps 1 --warmup 1 --no-cpu-baseline > gpurun_out/bench_coop2.json 2> gpurun_out/bench_coop2.err
echo "bench coop2 rc=$?"
