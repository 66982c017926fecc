set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1100 python3 tools/ab.py variants/dry0/librt_hip.so variants/dry16/librt_hip.so variants/dry64/librt_hip.so "variants/dry0/librt_hip.so@--share-of+8" "variants/dry16/librt_hip.so@--share-of+8" "variants/dry64/librt_hip.so@--share-of+8" --rounds 3 > gpurun_out/ab8.log 2>&1
echo "ab rc=$?"; tail -6 gpurun_out/ab8.log
