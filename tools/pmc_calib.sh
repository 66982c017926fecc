#!/bin/bash
# tools/pmc_calib.sh — what SQ_ACTIVE_INST_VALU and SQ_ACTIVE_INST_VALU2 ("quad-cycles two
# VALU instructions are issued": gfx950's dual issue) count: one rocprofv3 pass of
# the per-instruction microbenchmark kernels (known issue cost each) and of the c4
# megakernel with the same counters.  Output: gpurun_out/calib/.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/calib
mkdir -p $O
C="SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_VALU2 SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_THREAD_CYCLES_VALU SQ_WAVES SQ_ACTIVE_INST_ANY"
timeout -s KILL 120 rocprofv3 --pmc $C -d $O/micro -o run --output-format csv -- tools/microbench/valu_rates > $O/micro.log 2>&1
timeout -s KILL 240 rocprofv3 --pmc $C -d $O/c4 -o run --output-format csv -- python3 bench.py --config c4 --steps 1 --warmup 0 --no-cpu-baseline > $O/c4.log 2>&1
echo done
