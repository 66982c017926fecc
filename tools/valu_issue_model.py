#!/usr/bin/env python3
"""tools/valu_issue_model.py — issue-cycle demand of the megakernel on gfx950, from measurements.

The megakernel is bound by VALU issue, but gfx950's VALU
instructions do not all cost the same: tools/microbench/valu_rates.hip measures, with
8 independent chains per wave and 8 waves per SIMD, ~2.4 cycles per wave-instruction
for v_add/sub/mul_f32, v_add_u32, v_and/xor/or and v_mov_b32, ~4.2 for FMA, min/max,
compares, selects, shifts, integer multiplies, 64-bit and f64 operations, and ~8.2 for
transcendentals (profiles/r<NN>/valu_rates.log, cycles at the 2.4 GHz clock the
device reports).  A roof that charges every instruction 2 cycles understates the
VALU's load by ~1.7x; SQ_ACTIVE_INST_VALU charges every instruction one quad-cycle
(4 cycles, transcendentals 8: tools/pmc_calib.sh) and overstates it.

The model:
  * dynamic instruction counts per PMC class (SQ_INSTS_VALU_{ADD,MUL,FMA,TRANS}_F32,
    _INT32, _INT64, _CVT, _{ADD,MUL,FMA}_F64; the rest of SQ_INSTS_VALU is "other")
    of the timed launch (tools/pmc_classes.sh);
  * each class's cost = the mean measured cost of its opcodes, weighted by how often
    each opcode appears in the kernel's code object (static mix within the class —
    the one assumption; the class totals themselves are measured);
  * demand = sum(class count x class cost) cycles, over 1024 SIMDs.
frac = demand / (kernel time x the kernel's own clock, GRBM_GUI_ACTIVE / 8 / time of
the SQ pass): the share of the SIMDs' issue capacity the kernel's VALU instructions
need.  Costs are in cycles at the clock each microbenchmark kernel measured for itself.

usage: valu_issue_model.py RATES_LOG CLASSES_DIR OUT_JSON [ISA_S] [SAMPLES] [CONFIG] [CLOCK_GHZ]
  CLASSES_DIR holds pass1/ and pass2/ rocprofv3 outputs (tools/final_profile.sh);
  ISA_S = the device assembly (hipcc --cuda-device-only -S of rt_kernel.hip); built
  here when omitted.
"""
import collections
import csv
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "peter-shirley-ray-tracing-the-next-week_amd")
# the timed variant per config: <count, profile, width, features, mode>
SYMBOLS = {
    "c4": "_ZN12_GLOBAL__N_113rt_megakernelILb0ELb0ELi2ELi16ELi1EEEv12RtKernelArgs",   # final(): media only, LDS BVH2
    "c5": "_ZN12_GLOBAL__N_113rt_megakernelILb0ELb0ELi2ELi16ELi1EEEv12RtKernelArgs",
    "c3": "_ZN12_GLOBAL__N_113rt_megakernelILb0ELb0ELi2ELi12ELi1EEEv12RtKernelArgs",   # random_motion: checker + pre-scan
    "c2": "_ZN12_GLOBAL__N_113rt_megakernelILb0ELb0ELi2ELi1ELi2EEEv12RtKernelArgs",    # cornell_box: instances, flat scan
}
SYMBOL = SYMBOLS["c4"]
CLOCK_HZ = 2.4e9
SIMDS = 1024

# PMC class of an opcode (the microbenchmark kernels under rocprofv3 show which class
# counts which instruction: tools/pmc_classes.sh)
CLASSES = [
    ("SQ_INSTS_VALU_TRANS_F32", r"^v_(sqrt|rcp|rsq|exp|log|sin|cos|rcp_iflag)_f32$"),
    ("SQ_INSTS_VALU_ADD_F32", r"^v_(add|sub|subrev)_f32$|^v_pk_add_f32$"),
    ("SQ_INSTS_VALU_MUL_F32", r"^v_mul_f32$|^v_pk_mul_f32$"),
    ("SQ_INSTS_VALU_FMA_F32", r"^v_(fma|fmac|fmaak|fmamk|mad|mac)_f32$|^v_pk_fma_f32$|^v_div_fmas_f32$"),
    ("SQ_INSTS_VALU_CVT", r"^v_cvt_"),
    ("SQ_INSTS_VALU_ADD_F64", r"^v_add_f64$"),
    ("SQ_INSTS_VALU_MUL_F64", r"^v_mul_f64$"),
    ("SQ_INSTS_VALU_FMA_F64", r"^v_(fma|fmac)_f64$|^v_div_fmas_f64$"),
    ("SQ_INSTS_VALU_INT64", r"^v_mad_u64_u32$|^v_mad_i64_i32$|^v_lshl_add_u64$"),
    ("SQ_INSTS_VALU_INT32", r"^v_(add|sub|subrev)_(u32|i32)$|^v_(add|sub|subrev)_co_u32$|^v_(addc|subb|subbrev)_co_u32$"
                            r"|^v_mul_(lo|hi)_(u32|i32)$|^v_mul_(u32_u24|i32_i24|hi_u32_u24|hi_i32_i24)$"
                            r"|^v_mad_(u32_u24|i32_i24)$|^v_(max|min)_(i32|u32)$|^v_bfe_(u32|i32)$|^v_add3_u32$"),
]
FAST = re.compile(r"^v_(add|sub|subrev|mul)_f32$|^v_(add|sub|subrev)_(u32|i32)$|^v_(and|or|xor|not)_b32$|^v_mov_b32$")
TRANS = re.compile(r"^v_(sqrt|rcp|rsq|exp|log|sin|cos|rcp_iflag)_f(32|64)$")


def measured_costs(path):
    """opcode -> cycles per wave-instruction per SIMD (valu_rates.log)."""
    costs = {}
    for line in open(path):
        m = re.match(r"\s*(v_[a-z0-9_]+)(\s+\(sgpr mask\))?\s+[\d.]+ ms\s+([\d.]+) cycles", line)
        if not m:
            continue
        name, sgpr, cyc = m.group(1), m.group(2), float(m.group(3))
        # cycles at the clock the kernel measured itself (s_memtime / s_memrealtime), when sane
        mc = re.search(r"measured clock (\d+) MHz: ([\d.]+) cycles", line)
        if mc and 1500 <= int(mc.group(1)) <= 2600:
            cyc = float(mc.group(2))
        if name == "v_cndmask_b32" and not sgpr:
            continue   # the VCC-mask form measured a hazard of the harness, not the issue cost
        costs[name] = cyc
    return costs


def cost_of(op, costs):
    if op in costs:
        return costs[op]
    if op.endswith("_e32") or op.endswith("_e64"):
        op = op[:-4]
    if op in costs:
        return costs[op]
    if TRANS.match(op):
        return costs.get("v_sqrt_f32", 8.2)
    if FAST.match(op):
        return costs.get("v_add_f32", 2.4)
    return costs.get("v_fma_f32", 4.2) if op.startswith("v_fma") else costs.get("v_min3_f32", 4.2)


def static_opcodes(isa_path, symbol):
    ops = collections.Counter()
    inside = False
    for line in open(isa_path):
        if line.startswith(symbol + ":"):
            inside = True
            continue
        if inside and "s_endpgm" in line:
            break
        if inside:
            m = re.match(r"\s+(v_[a-z0-9_]+)", line)
            if m:
                op = re.sub(r"_(e32|e64|sdwa|dpp)$", "", m.group(1))
                ops[op] += 1
    return ops


def class_of(op):
    for name, rx in CLASSES:
        if re.match(rx, op):
            return name
    return "other"


def pmc_counts(classes_dir):
    tot = {}
    for sub in ("pass1", "pass2"):   # rocprofv3 output dirs, or the copies committed under profiles/
        path = os.path.join(classes_dir, sub, "run_counter_collection.csv")
        if not os.path.exists(path):
            path = os.path.join(classes_dir, "pmc_classes_%s.csv" % sub[-1])
        first = None   # the first timed launch (c5 on one GPU: two launches of different sizes)
        for r in csv.DictReader(open(path)):
            if "rt_megakernel<false, false" not in r["Kernel_Name"]:
                continue
            first = r["Dispatch_Id"] if first is None else first
            if r["Dispatch_Id"] != first:
                continue
            tot[r["Counter_Name"]] = float(r["Counter_Value"])
            tot["kernel_ns_" + sub] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return tot


def build_isa():
    out = os.path.join(tempfile.mkdtemp(), "rt_kernel.s")
    subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
                    "-I" + os.path.join(ROOT, "include"), "-I" + os.path.join(PKG, "csrc"),
                    "-I" + os.path.join(PKG, "csrc", "host"), "-I" + os.path.join(PKG, "csrc", "hip"),
                    "--offload-arch=gfx950", "-munsafe-fp-atomics", "--cuda-device-only", "-S",
                    os.path.join(PKG, "csrc", "hip", "rt_kernel.hip"), "-o", out], check=True, capture_output=True)
    return out


def main():
    rates, classes_dir, out_json = sys.argv[1], sys.argv[2], sys.argv[3]
    isa = sys.argv[4] if len(sys.argv) > 4 and sys.argv[4] else build_isa()
    samples = float(sys.argv[5]) if len(sys.argv) > 5 else 250e6
    config = sys.argv[6] if len(sys.argv) > 6 else "c4"
    clock_hz = float(sys.argv[7]) * 1e9 if len(sys.argv) > 7 and sys.argv[7] else CLOCK_HZ
    symbol = SYMBOLS[config.split("_n")[0]]   # c5_nN: a rank's share of c5, the same kernel
    costs = measured_costs(rates)
    ops = static_opcodes(isa, symbol)
    per_class = collections.defaultdict(lambda: [0, 0.0])   # static count, static count x cost
    for op, n in ops.items():
        c = class_of(op)
        per_class[c][0] += n
        per_class[c][1] += n * cost_of(op, costs)
    pmc = pmc_counts(classes_dir)
    total = pmc["SQ_INSTS_VALU"]
    dyn = {name: pmc[name] for name, _ in CLASSES}
    dyn["other"] = total - sum(dyn.values())
    demand = 0.0
    rows = {}
    for c, n in dyn.items():
        sc, sw = per_class.get(c, [0, 0.0])
        avg = sw / sc if sc else costs.get("v_min3_f32", 4.2)
        demand += n * avg
        rows[c] = {"count_per_launch": n, "count_per_sample": n / samples, "cycles_each": avg, "static_opcodes": sc}
    kernel_ns = pmc["kernel_ns_pass1"]
    cap = SIMDS * clock_hz * kernel_ns * 1e-9
    res = {
        "model": "sum over PMC classes of (dynamic count x static-mix mean of the measured per-opcode issue cost)",
        "clock_hz": clock_hz, "simds": SIMDS, "samples_per_launch": samples,
        "valu_insts_per_launch": total, "valu_issue_cycles_per_launch": demand,
        "valu_issue_cycles_per_sample": demand / samples,
        "kernel_ns_pmc_pass": kernel_ns,
        "valu_issue_frac_pmc_pass": demand / cap,
        "uniform_2cyc_frac": total * 2 / cap, "uniform_4cyc_frac": total * 4 / cap,
        "classes": rows, "costs_measured": costs,
        "isa_symbol": symbol, "config": config,
    }
    with open(out_json, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps({k: v for k, v in res.items() if k not in ("classes", "costs_measured")}, indent=1))
    for c, r in rows.items():
        print(f"{c:26s} {r['count_per_launch']:.3e}  x {r['cycles_each']:.2f} cyc  (static opcodes {r['static_opcodes']})")


if __name__ == "__main__":
    main()
