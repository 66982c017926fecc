#!/usr/bin/env python3
"""tools/lanes_summary.py OUTDIR [OUT.json] — VALU lane utilisation of the timed
megakernel per config from the `lanes_<cfg>` rocprofv3 passes of tools/gpu_session.sh
(SQ_THREAD_CYCLES_VALU / (64 x SQ_ACTIVE_INST_VALU): the share of the 64 lanes that
are active in the issued VALU slots; the method of profiles/r01/lane_utilisation.txt)."""
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
    res = {"method": "SQ_THREAD_CYCLES_VALU / (64 * SQ_ACTIVE_INST_VALU), first dispatch of the timed megakernel",
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
        v = first_dispatch(csvs[0])
        if "SQ_THREAD_CYCLES_VALU" in v and v.get("SQ_ACTIVE_INST_VALU"):
            v["lane_utilisation"] = v["SQ_THREAD_CYCLES_VALU"] / (64 * v["SQ_ACTIVE_INST_VALU"])
        res["configs"][os.path.basename(d)[len("lanes_"):]] = v
    text = json.dumps(res, indent=1)
    print(text)
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            f.write(text + "\n")


if __name__ == "__main__":
    main()
