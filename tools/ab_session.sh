# tools/ab_session.sh — one A/B session on the gpurun box (edit the variants): parity tests with
# one variant library, then tools/ab.py over the variants (c4; @--config+c3 for c3).
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
RTNW_LIB=$PWD/variants/sdpk/librt_hip.so timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -q --timeout 300 --timeout-method thread -x > gpurun_out/t14.log 2>&1
echo "tests rc=$?"; tail -2 gpurun_out/t14.log
timeout -k 10 900 python3 tools/ab.py variants/nopk/librt_hip.so variants/pk/librt_hip.so variants/sd/librt_hip.so variants/sdpk/librt_hip.so "variants/nopk/librt_hip.so@--config+c3" "variants/pk/librt_hip.so@--config+c3" "variants/sdpk/librt_hip.so@--config+c3" --rounds 3 > gpurun_out/ab14.log 2>&1
echo "ab rc=$?"; tail -4 gpurun_out/ab14.log
