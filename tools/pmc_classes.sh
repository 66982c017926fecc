#!/bin/bash
# tools/pmc_classes.sh — VALU instruction classes (SQ_INSTS_VALU_*) of the timed c4
# megakernel and of the per-instruction microbenchmark kernels (which class each
# instruction is counted in), two rocprofv3 passes each.  Output: gpurun_out/classes/.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/classes
mkdir -p $O
P1="SQ_INSTS_VALU SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_INT64 SQ_INSTS_VALU_CVT"
P2="SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH"
B="python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline"
i=0
for ctrs in "$P1" "$P2"; do
  i=$((i+1))
  echo "== micro pass $i"
  timeout -s KILL 120 rocprofv3 --pmc $ctrs -d $O/micro$i -o run --output-format csv -- tools/microbench/valu_rates > $O/micro$i.log 2>&1
  echo "== c4 pass $i"
  timeout -s KILL 240 rocprofv3 --pmc $ctrs -d $O/c4_$i -o run --output-format csv -- $B > $O/c4_$i.log 2>&1
done
echo done
