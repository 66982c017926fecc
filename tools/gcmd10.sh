set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
L=variants/cur/librt_hip.so
timeout -k 10 1100 python3 tools/ab.py $L $L:RTNW_SAH_TRAV=0.6 $L:RTNW_SAH_TRAV=0.8 $L:RTNW_SAH_TRAV=1.3 $L:RTNW_SAH_TRAV=1.7 --rounds 3 > gpurun_out/ab10.log 2>&1
echo "ab rc=$?"; tail -5 gpurun_out/ab10.log
