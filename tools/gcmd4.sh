set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
RTNW_LIB=$PWD/variants/kre/librt_hip.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread -k "bvh_widths or feature_variants or gpu_matches_oracle" > gpurun_out/t4.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/t4.log
timeout -k 10 1000 python3 tools/ab.py variants/base/librt_hip.so variants/kre/librt_hip.so "variants/base/librt_hip.so@--config+c3" "variants/kre/librt_hip.so@--config+c3" "variants/base/librt_hip.so@--config+c2" "variants/kre/librt_hip.so@--config+c2" --rounds 3 > gpurun_out/ab4.log 2>&1
echo "ab rc=$?"; tail -6 gpurun_out/ab4.log
