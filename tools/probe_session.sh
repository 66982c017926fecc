set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 600 python3 tools/scaling_probe.py --out gpurun_out/scaling_probe.json > gpurun_out/scaling_probe.log 2>&1
echo "probe rc=$?"; tail -3 gpurun_out/scaling_probe.log
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/gpu_tests_final.log 2>&1
echo "tests rc=$?"; tail -1 gpurun_out/gpu_tests_final.log
