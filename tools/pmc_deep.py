#!/usr/bin/env python3
"""tools/pmc_deep.py OUTDIR — prints the counters of the pmc_d* passes (tools/gpu_session.sh
pmc_deep) for the timed megakernel, with per-wave-cycle and per-cycle ratios.  Diagnostic."""
import csv
import glob
import os
import sys

KERNEL = os.environ.get("RT_PMC_KERNEL", "rt_megakernel<false, false")
vals = {}
for path in sorted(glob.glob(os.path.join(sys.argv[1], "pmc_d*", "run_counter_collection.csv"))):
    seen = None
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL not in r["Kernel_Name"]:
                continue
            if seen is None:
                seen = r["Dispatch_Id"]
                vals.setdefault("dur_ns", int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
            if r["Dispatch_Id"] == seen:
                vals[r["Counter_Name"]] = float(r["Counter_Value"])
for k in sorted(vals):
    print(f"{k:36s} {vals[k]:.6g}")
wc = vals.get("SQ_WAVE_CYCLES")
if wc:
    print("-- per wave-cycle")
    for k in sorted(vals):
        if k.startswith("SQ_ACTIVE") or k.startswith("SQ_WAIT"):
            print(f"{k:36s} {vals[k] / wc:.4f}")
g = vals.get("GRBM_GUI_ACTIVE")
if g:
    cyc = g / 8   # GRBM counts per XCD
    print(f"-- cycles (GRBM/8) {cyc:.4g}")
    for k in ("TA_TA_BUSY", "TD_TD_BUSY", "SQC_ICACHE_BUSY_CYCLES", "TCP_PENDING_STALL_CYCLES"):
        if k in vals:
            print(f"{k:36s} per CU-cycle {vals[k] / cyc / 256:.4f}")
if "SQC_ICACHE_REQ" in vals:
    print("icache miss rate", vals.get("SQC_ICACHE_MISSES", 0) / max(1, vals["SQC_ICACHE_REQ"]))
if "SQ_THREAD_CYCLES_VALU" in vals and "SQ_ACTIVE_INST_VALU" in vals:
    print("VALU lane utilization", vals["SQ_THREAD_CYCLES_VALU"] / (64 * vals["SQ_ACTIVE_INST_VALU"]))
if "TCP_TOTAL_CACHE_ACCESSES" in vals:
    print("L1 miss rate", vals.get("TCP_CACHE_MISS", 0) / max(1, vals["TCP_TOTAL_CACHE_ACCESSES"]))
