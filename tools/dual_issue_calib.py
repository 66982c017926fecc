#!/usr/bin/env python3
"""tools/dual_issue_calib.py CALIB_DIR OUT.json — checks the measured VALU issue model on the
per-opcode microbenchmark (tools/pmc_calib.sh output: CALIB_DIR/micro.log with the timed
cycles per wave-instruction, CALIB_DIR/micro/*counter_collection.csv with the counters).

Model: the VALU issues one wave64 instruction per quad-cycle (SQ_ACTIVE_INST_VALU counts one
per instruction, two per transcendental), two in one quad-cycle when they dual-issue
(SQ_ACTIVE_INST_VALU2 counts those quad-cycles), so an instruction costs
  4 x (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SQ_INSTS_VALU   cycles.
Per opcode the table holds the prediction, the timed cycles (at the clock the kernel
measured for itself) and their difference, which is the microbenchmark loop's own SALU and
branch overhead (~13 cycles per 32 VALU instructions)."""
import collections
import csv
import glob
import json
import re
import sys


def main():
    d, out = sys.argv[1], sys.argv[2]
    timed = {}
    names = []
    for line in open(f"{d}/micro.log"):
        m = re.match(r"(v_[a-z0-9_]+(?: \([a-z ,]+\))?)\s+[\d.]+ ms .*measured clock (\d+) MHz: ([\d.]+) cycles", line)
        if m:
            timed[m.group(1)] = float(m.group(3))
            names.append(m.group(1))
    rows = list(csv.DictReader(open(glob.glob(f"{d}/micro/**/*counter_collection.csv", recursive=True)[0])))
    by = collections.OrderedDict()
    for r in rows:
        k = r["Kernel_Name"].split("(")[0]
        if k.startswith("__amd"):
            continue
        by.setdefault(k, collections.OrderedDict()).setdefault(r["Dispatch_Id"], {})[r["Counter_Name"]] = \
            float(r["Counter_Value"])
    res = {"model": "cycles per wave64 VALU instruction = 4 (SQ_ACTIVE_INST_VALU - SQ_ACTIVE_INST_VALU2) / SQ_INSTS_VALU",
           "opcodes": {}}
    # label -> kernel, from the microbenchmark's own table ({"label", kernel} pairs)
    import os
    src = open(os.path.join(os.path.dirname(os.path.abspath(__file__)), "microbench", "valu_rates.hip")).read()
    kern_of = dict(re.findall(r'\{"([^"]+)", (k_[a-z0-9_]+)\}', src))
    for name in names:
        kern = kern_of.get(name)
        if kern not in by:
            continue
        v = next(iter(by[kern].values()))
        i, a, a2 = v["SQ_INSTS_VALU"], v["SQ_ACTIVE_INST_VALU"], v["SQ_ACTIVE_INST_VALU2"]
        pred = 4 * (a - a2) / i
        res["opcodes"][name] = {"kernel": kern, "active_per_inst": a / i, "dual_quads_per_inst": a2 / i,
                                "predicted_cycles": pred, "timed_cycles": timed[name],
                                "timed_minus_predicted": timed[name] - pred}
    diffs = [o["timed_minus_predicted"] for n, o in res["opcodes"].items() if n != "v_cndmask_b32"]
    res["loop_overhead_cycles_per_instr"] = {"min": min(diffs), "max": max(diffs), "mean": sum(diffs) / len(diffs)}
    res["note"] = ("v_cndmask_b32 with the VCC mask written by an SALU move times ~23 cycles but counts one quad-cycle: "
                   "a pipeline interlock of the harness (SALU-written VCC read by the VALU), not issue; the "
                   "megakernel's selects read compare results and cost what the SGPR-mask form does")
    json.dump(res, open(out, "w"), indent=1)
    for n, o in res["opcodes"].items():
        print(f"{n:36s} A/I {o['active_per_inst']:.3f} A2/I {o['dual_quads_per_inst']:.3f} "
              f"predicted {o['predicted_cycles']:.2f}  timed {o['timed_cycles']:.2f}")
    print(res["loop_overhead_cycles_per_instr"])


if __name__ == "__main__":
    main()
