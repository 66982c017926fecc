set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -rA > gpurun_out/gpu_tests.log 2>&1
echo "tests rc=$?"; tail -3 gpurun_out/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
echo "smoke rc=$?"; tail -2 gpurun_out/smoke.log
for c in c5_n2 c5_n4; do
  timeout -k 10 500 bash tools/final_profile.sh $c > gpurun_out/final_profile_$c.log 2>&1
  rc=$?; echo "profile $c rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
