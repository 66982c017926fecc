# tools/ab_session.sh — one A/B session on the gpurun box (edit the variants): tools/ab.py over
# libraries / environment settings (c4; @--config+c3 for c3, @--share-of+8 for a c5 rank share).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
L=variants/cur/librt_hip.so
timeout -k 10 1100 python3 tools/ab.py $L $L:RTNW_TAIL_CLAIMS=16 $L:RTNW_TAIL_CLAIMS=64 $L:RTNW_TAIL_CLAIMS=128 $L:RTNW_CLAIM=4 $L:RTNW_CLAIM=16 "$L@--share-of+8" "$L:RTNW_TAIL_CLAIMS=64@--share-of+8" "$L:RTNW_TAIL_CLAIMS=128@--share-of+8" --rounds 3 > gpurun_out/ab15.log 2>&1
echo "ab rc=$?"; grep SUMMARY gpurun_out/ab15.log
