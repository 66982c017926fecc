# tools/round_profile.sh — the round's PMC evidence on the gpurun box: tools/final_profile.sh for each config
# in PROF_CFGS (default c4, c5_n8, c5, c3, c2); summarise on the host with tools/pmc_traffic.py
# and tools/lanes_summary.py.
set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
for c in ${PROF_CFGS:-c4 c5_n8 c5 c3 c2}; do
  timeout -k 10 500 bash tools/final_profile.sh $c > gpurun_out/final_profile_$c.log 2>&1
  rc=$?; echo "profile $c rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
