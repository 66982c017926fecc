#!/usr/bin/env python3
"""tools/lanes_summary.py OUTDIR [OUT.json] — VALU lane utilisation and VALU issue cost of the
timed megakernel per config from the `lanes_<cfg>` rocprofv3 passes (tools/final_profile.sh):

  lane_utilisation = SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU): the share of the 64
    lanes active in the issued VALU slots (the method of profiles/r01/lane_utilisation.txt);
  issue_cycles_per_instr = 4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SQ_INSTS_VALU:
    the SIMD cycles the VALU spends per wave-instruction, MEASURED.  gfx950 issues a
    wave64 VALU instruction in one quad-cycle (SQ_ACTIVE_INST_VALU counts one per
    instruction, two per transcendental) and can issue two in one quad-cycle
    (SQ_ACTIVE_INST_VALU2 counts those quad-cycles): f32 add/sub/mul, v_mov, logic, integer
    add and f32 FMA with three distinct source registers pair up; min/max, compares,
    selects, shifts, packed and 64-bit operations do not (tools/pmc_calib.sh,
    profiles/r05/valu_dual_issue.json).  This replaces round 4's static-mix model of
    tools/valu_issue_model.py, which charged 45 % of the instructions an assumed cost."""
import csv
import glob
import json
import os
import sys

KERNEL = os.environ.get("RT_PMC_KERNEL", "rt_megakernel<false, false")


def first_dispatch(path):
    vals, seen = {}, None
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL not in r["Kernel_Name"]:
                continue
            if seen is None:
                seen = r["Dispatch_Id"]
                vals["kernel"] = r["Kernel_Name"]
                vals["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
                vals["scratch_bytes_per_lane"] = int(r["Scratch_Size"])
            if r["Dispatch_Id"] == seen:
                vals[r["Counter_Name"]] = float(r["Counter_Value"])
    return vals


def main():
    out = sys.argv[1]
    res = {"method": "lane_utilisation = SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU); issue_cycles_per_instr = "
                     "4 * (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SQ_INSTS_VALU; first dispatch of the timed megakernel",
           "configs": {}}
    # the device code object the passes ran (bench.py matches a profile to its library by it)
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    try:
        import bench
        res["kernel_sha16"] = bench.kernel_sha16(os.environ.get("RTNW_LIB") or None)
    except Exception as e:   # noqa: BLE001 (diagnostic tool: record why)
        res["kernel_sha16_error"] = repr(e)
    for d in sorted(glob.glob(os.path.join(out, "lanes_c*"))):
        csvs = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
        if not csvs:
            continue
        rec = os.path.join(d, "kernel_sha16.txt")   # tools/final_profile.sh: the build the passes ran
        if os.path.exists(rec) and open(rec).read().strip() != res.get("kernel_sha16"):
            print(f"{d}: counters of kernel {open(rec).read().strip()}, not this library's: skipped", file=sys.stderr)
            continue
        v = first_dispatch(csvs[0])
        if "SQ_THREAD_CYCLES_VALU" in v and v.get("SQ_ACTIVE_INST_VALU"):
            v["lane_utilisation"] = v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"])
        if "SQ_ACTIVE_INST_VALU2" in v and v.get("SQ_INSTS_VALU"):
            v["dual_issue_share"] = 2 * v["SQ_ACTIVE_INST_VALU2"] / v["SQ_INSTS_VALU"]   # instructions issued in pairs
            v["issue_cycles_per_instr"] = 4 * (v["SQ_ACTIVE_INST_VALU"] - v["SQ_ACTIVE_INST_VALU2"]) / v["SQ_INSTS_VALU"]
        res["configs"][os.path.basename(d)[len("lanes_"):]] = v
    text = json.dumps(res, indent=1)
    print(text)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
