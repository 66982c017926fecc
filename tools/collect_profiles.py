#!/usr/bin/env python3
"""tools/collect_profiles.py OUT PROFILE_DIR — copies the summaries of a
`tools/gpu_session.sh prof pmc pmc_lanes stages stages_cornell` run (merged back
into OUT, normally gpurun_out/) into PROFILE_DIR (profiles/rNN/):
  kernel_stats_c4_1000spp.csv   rocprofv3 --kernel-trace --stats of bench.py
  kernel_trace_megakernel.csv   the megakernel's dispatches from the same run
  pmc_{fetch,write,l2,sq}_counters.csv, traffic.json, pmc_summary.md (tools/pmc_traffic.py)
  lane_utilisation.txt          SQ_THREAD_CYCLES_VALU / (64 SQ_ACTIVE_INST_VALU), both engines
  stage_profile_{final,cornell}.json
Missing inputs are skipped."""
import csv
import json
import os
import shutil
import subprocess
import sys

out, prof = sys.argv[1], sys.argv[2]
os.makedirs(prof, exist_ok=True)
here = os.path.dirname(os.path.abspath(__file__))


def cp(src, dst):
    s = os.path.join(out, src)
    if os.path.exists(s):
        shutil.copy(s, os.path.join(prof, dst))


cp("prof/run_kernel_stats.csv", "kernel_stats_c4_1000spp.csv")
trace = os.path.join(out, "prof/run_kernel_trace.csv")
if os.path.exists(trace):
    with open(trace) as f, open(os.path.join(prof, "kernel_trace_megakernel.csv"), "w") as g:
        for i, line in enumerate(f):
            if i == 0 or "rt_megakernel" in line:
                g.write(line)
for k in ("fetch", "write", "l2", "sq"):
    cp(f"pmc_{k}/run_counter_collection.csv", f"pmc_{k}_counters.csv")
subprocess.run([sys.executable, os.path.join(here, "pmc_traffic.py"), out, prof], check=False,
               stdout=subprocess.DEVNULL)


def lanes(path):
    d = {}
    if not os.path.exists(path):
        return d
    with open(path) as f:
        for r in csv.DictReader(f):
            n = r["Kernel_Name"]
            if "rt_megakernel<false, false" not in n:
                continue
            if d and r["Dispatch_Id"] != d["id"]:
                continue   # the first timed dispatch only
            d["id"] = r["Dispatch_Id"]
            d[r["Counter_Name"]] = float(r["Counter_Value"])
            d["dur_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return d


lines = ["# VALU lane utilisation (SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU), bench.py --spp 128"]
for name, sub in (("megakernel", "pmc_l1"),):
    d = lanes(os.path.join(out, sub, "run_counter_collection.csv"))
    if not d:
        continue
    lines.append("## " + name)
    for k in ("SQ_ACTIVE_INST_VALU", "SQ_INSTS_VALU", "SQ_THREAD_CYCLES_VALU", "dur_ns"):
        lines.append(f"{k:36s} {d[k]:.6g}")
    lines.append(f"VALU lane utilization {d['SQ_THREAD_CYCLES_VALU'] / (64 * d['SQ_ACTIVE_INST_VALU'])}")
if len(lines) > 1:
    with open(os.path.join(prof, "lane_utilisation.txt"), "w") as f:
        f.write("\n".join(lines) + "\n")

for log, name in (("stages.log", "stage_profile_final.json"), ("stages_cornell.log", "stage_profile_cornell.json")):
    p = os.path.join(out, log)
    if os.path.exists(p):
        s = open(p).read()
        j = json.loads(s[s.index("{"):])
        with open(os.path.join(prof, name), "w") as f:
            json.dump(j, f, indent=1)
        print(name, j["plain_kernel_ms"], {k: round(v, 3) for k, v in j["stage_share"].items()})
print("\n".join(lines))
