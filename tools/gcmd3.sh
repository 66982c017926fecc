set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
for v in basecnt coopcnt coop2cnt; do
  RTNW_LIB=$PWD/variants/$v/librt_hip.so timeout -k 10 300 python3 tools/stage_profile.py final > gpurun_out/stage_$v.json 2> gpurun_out/stage_$v.err
  echo "stage $v rc=$?"
done
