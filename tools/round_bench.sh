# tools/round_bench.sh — the round's bench evidence on the gpurun box: tools/final_bench.sh (kernel
# trace + bench lines), the c4 wave timeline and the final() stage profile.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
timeout -k 10 900 bash tools/final_bench.sh > gpurun_out/final_bench.log 2>&1
rc=$?; echo "final_bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/wave_log.py --config c4 --out gpurun_out/wave_log_c4.json > gpurun_out/wave_log_c4.log 2>&1
echo "wave_log rc=$?"
timeout -k 10 300 python3 tools/stage_profile.py final > gpurun_out/stage_final.json 2> gpurun_out/stage_final.err
echo "stage rc=$?"
