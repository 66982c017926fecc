set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
RTNW_LIB=$PWD/variants/sd/librt_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -x > gpurun_out/t13.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/t13.log
timeout -k 10 900 python3 tools/ab.py variants/cur/librt_hip.so variants/sd/librt_hip.so "variants/cur/librt_hip.so@--config+c3" "variants/sd/librt_hip.so@--config+c3" "variants/cur/librt_hip.so@--config+c2" "variants/sd/librt_hip.so@--config+c2" --rounds 3 > gpurun_out/ab13.log 2>&1
echo "ab rc=$?"; tail -6 gpurun_out/ab13.log
