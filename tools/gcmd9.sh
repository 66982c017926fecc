set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 1100 python3 tools/ab.py variants/cur/librt_hip.so variants/ifcvt/librt_hip.so variants/trk/librt_hip.so variants/prio/librt_hip.so variants/relax/librt_hip.so variants/nounc/librt_hip.so variants/liver/librt_hip.so --rounds 3 > gpurun_out/ab9.log 2>&1
echo "ab rc=$?"; tail -7 gpurun_out/ab9.log
