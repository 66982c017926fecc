set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/t6.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/t6.log
timeout -k 10 600 python3 tools/ab.py variants/kre/librt_hip.so variants/med/librt_hip.so --rounds 3 > gpurun_out/ab6.log 2>&1
echo "ab rc=$?"; tail -2 gpurun_out/ab6.log
