set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1100 python3 tools/ab.py variants/med/librt_hip.so variants/rb44/librt_hip.so variants/rb52/librt_hip.so variants/dt6/librt_hip.so variants/dt10/librt_hip.so variants/ds3/librt_hip.so --rounds 3 > gpurun_out/ab7.log 2>&1
echo "ab rc=$?"; tail -6 gpurun_out/ab7.log
