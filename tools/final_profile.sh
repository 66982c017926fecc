#!/bin/bash
# tools/final_profile.sh — the round's evidence for the library in the tree, on the
# gpurun box: PMC passes of the timed c4 megakernel (separate rocprofv3 passes: HBM
# bytes, L2, SQ occupancy/waits, and the two VALU instruction-class passes), the
# per-instruction issue-cost microbenchmark.  Every step under its own time limit;
# the first failure ends the script.  Then, on the build host, the summary
# (traffic.json with the issue-weighted VALU model, which bench.py's roofline reads):
#   python3 tools/pmc_traffic.py gpurun_out/final_c4 profiles/r<NN> 250000000 c4
# (c2 / c3 / c5: profiles/r<NN>/<cfg>, samples per launch 32e6 / 160e6 / 500e6 — c5
# on one GPU runs as two sample batches)
# and back on the box tools/final_bench.sh (kernel trace + bench lines).
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
CFG=${1:-c4}   # the bench config profiled (c4 = the metric's; c2, c3, c5 for their own bench lines;
               # c5_nN: one rank's share of c5 split over N GPUs, bench.py --share-of N)
O=gpurun_out/final_$CFG
mkdir -p $O/classes gpurun_out/lanes_$CFG
# the device code these passes run: the host-side summaries refuse counters of another build
python3 -c "import bench; print(bench.kernel_sha16())" | tee $O/kernel_sha16.txt > gpurun_out/lanes_$CFG/kernel_sha16.txt
case $CFG in
  c5_n*) B="python3 bench.py --share-of ${CFG#c5_n} --steps 1 --warmup 0 --no-cpu-baseline" ;;
  *)     B="python3 bench.py --config $CFG --steps 1 --warmup 0 --no-cpu-baseline" ;;
esac
for pass in "FETCH_SIZE:fetch" "WRITE_SIZE:write" "TCC_HIT_sum TCC_MISS_sum:l2" \
            "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE:sq"; do
  ctrs=${pass%%:*}; name=${pass##*:}
  echo "== pmc $name"
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $O/pmc_$name -o run --output-format csv -- $B > $O/pmc_$name.log 2>&1
done
echo "== pmc lds"   # LDS bank / address conflicts and waits
timeout -s KILL 240 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_LDS SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_WAVE_CYCLES \
    -d $O/pmc_lds -o run --output-format csv -- $B > $O/pmc_lds.log 2>&1
echo "== pmc lanes"   # VALU lane utilisation (tools/lanes_summary.py reads gpurun_out/lanes_<cfg>)
timeout -s KILL 240 rocprofv3 --pmc SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_INSTS_VALU -d gpurun_out/lanes_$CFG -o run \
    --output-format csv -- $B > $O/pmc_lanes.log 2>&1
i=0
for ctrs in "SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT" \
            "SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH"; do
  i=$((i+1))
  echo "== pmc classes $i"
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $O/classes/pass$i -o run --output-format csv -- $B > $O/classes/pass$i.log 2>&1
done
if [ "$CFG" = c4 ]; then
  echo "== microbenchmark"
  timeout -k 10 120 tools/microbench/valu_rates > $O/valu_rates.log 2>&1
fi
echo done
