set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bvh_widths or feature_variants or gpu_matches_oracle or medium_size or claim_size or tile or baseline_configs" > gpurun_out/t1.log 2>&1
echo "tests rc=$?"; tail -5 gpurun_out/t1.log
timeout -k 10 900 python3 tools/ab.py variants/base/librt_hip.so variants/coop/librt_hip.so "variants/base/librt_hip.so@--config+c3" "variants/coop/librt_hip.so@--config+c3" --rounds 3 > gpurun_out/ab1.log 2>&1
echo "ab rc=$?"; tail -6 gpurun_out/ab1.log
for v in coop; do
RTNW_LIB=variants/$v/librt_hip.so timeout -k 10 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/bench_$v.json 2> gpurun_out/bench_$v.err
echo "bench $v rc=$?"
done
