#!/usr/bin/env python3
"""tools/pmc_traffic.py OUTDIR PROFILE_DIR [SAMPLES] [CONFIG] — summarises rocprofv3 PMC passes of bench.py.

With OUTDIR/classes/ (tools/pmc_classes.sh) and the microbenchmark costs
(profiles/r<NN>/valu_rates.log, env RT_VALU_RATES), it also adds the issue-weighted
VALU model of tools/valu_issue_model.py (run on the build host: it compiles the
kernel's assembly for the static opcode mix).

Reads OUTDIR/pmc_{fetch,write,l2,sq}/run_counter_collection.csv (separate passes, as
MI355X_MICROARCH.md §rocprofv3 requires: FETCH_SIZE and WRITE_SIZE do not fit one
pass), keeps the dispatches of the timed megakernel (rt_megakernel<false, false>),
and writes:
  PROFILE_DIR/traffic.json  hbm_bytes_per_launch / _per_sample for bench.py's roofline
  PROFILE_DIR/pmc_summary.md
bench.py reads traffic.json for its roofline: VALU instructions per sample (the
binding roof: wave-level SQ_INSTS_VALU, each 2 cycles on a SIMD-32), HBM bytes per
sample, and lib_sha16 = the librt_hip.so build the counters were taken on.
HBM bytes = (2 x FETCH_SIZE + WRITE_SIZE) x 1024: FETCH_SIZE/WRITE_SIZE are in KiB and
gfx950's FETCH_SIZE reports half the bytes of wide reads (MI355X_MICROARCH.md §HBM);
the doubling is uncalibrated for this kernel's scattered 16-B reads, so the read
side is an upper estimate.
"""
import csv
import hashlib
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
KERNEL = os.environ.get("RT_PMC_KERNEL", "rt_megakernel<false, false")


def load(path):
    rows = {}
    if not os.path.exists(path):
        return rows
    with open(path) as f:
        for r in csv.DictReader(f):
            if KERNEL not in r["Kernel_Name"]:
                continue
            d = rows.setdefault(r["Dispatch_Id"], {"dur_ns": int(r["End_Timestamp"]) - int(r["Start_Timestamp"]),
                                                   "grid": int(r["Grid_Size"]), "vgpr": int(r["VGPR_Count"]),
                                                   "scratch": int(r["Scratch_Size"])})
            d[r["Counter_Name"]] = float(r["Counter_Value"])
    return rows


def first(rows):
    return next(iter(rows.values())) if rows else {}


def main():
    out, prof = sys.argv[1], sys.argv[2]
    samples = float(sys.argv[3]) if len(sys.argv) > 3 else 500 * 500 * 1000
    config = sys.argv[4] if len(sys.argv) > 4 else "c4"
    fetch = first(load(os.path.join(out, "pmc_fetch", "run_counter_collection.csv")))
    write = first(load(os.path.join(out, "pmc_write", "run_counter_collection.csv")))
    l2 = first(load(os.path.join(out, "pmc_l2", "run_counter_collection.csv")))
    sq = first(load(os.path.join(out, "pmc_sq", "run_counter_collection.csv")))
    lib = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                       "peter-shirley-ray-tracing-the-next-week_amd", "librt_hip.so")
    with open(lib, "rb") as f:
        sha = hashlib.sha256(f.read()).hexdigest()[:16]
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    ksha = bench.kernel_sha16(lib)
    # counters taken on another build (a stale gpurun_out/ directory) are not this library's
    rec = os.path.join(out, "kernel_sha16.txt")
    if os.path.exists(rec) and open(rec).read().strip() != ksha:
        print(f"{out}: counters of kernel {open(rec).read().strip()}, the library here is {ksha}: not summarised",
              file=sys.stderr)
        sys.exit(3)
    res = {"config": config, "workload": f"{config} (bench.py --config {config})", "samples_per_launch": samples,
           "lib_sha16": sha, "kernel_sha16": ksha}
    if fetch and write:
        fb = fetch["FETCH_SIZE"] * 1024.0
        wb = write["WRITE_SIZE"] * 1024.0
        res.update(fetch_size_bytes=fb, write_size_bytes=wb, hbm_bytes_per_launch=2 * fb + wb,
                   hbm_bytes_per_sample=(2 * fb + wb) / samples, kernel_ns=fetch["dur_ns"])
    if l2:
        res["l2_hit_rate"] = l2["TCC_HIT_sum"] / (l2["TCC_HIT_sum"] + l2["TCC_MISS_sum"])
    if sq:
        res["valu_active_per_wave_cycle"] = sq["SQ_ACTIVE_INST_VALU"] / sq["SQ_WAVE_CYCLES"]
        res["wait_any_per_wave_cycle"] = sq["SQ_WAIT_ANY"] / sq["SQ_WAVE_CYCLES"]
        res["wait_inst_any_per_wave_cycle"] = sq["SQ_WAIT_INST_ANY"] / sq["SQ_WAVE_CYCLES"]
        res["valu_insts_per_launch"] = sq["SQ_INSTS_VALU"]
        res["valu_insts_per_sample"] = sq["SQ_INSTS_VALU"] / samples   # wave-level instructions
        if "SQ_INSTS_SALU" in sq:
            res["salu_insts_per_sample"] = sq["SQ_INSTS_SALU"] / samples
        res["valu_issue_frac"] = sq["SQ_INSTS_VALU"] * 2 / (1024 * 2.4e9 * sq["dur_ns"] * 1e-9)
        res["valu_issue_frac_at_measured_clock"] = sq["SQ_INSTS_VALU"] * 2 / (1024 * sq["GRBM_GUI_ACTIVE"] / 8)
        res["kernel_ns_sq_pass"] = sq["dur_ns"]
        res["effective_clock_ghz"] = sq["GRBM_GUI_ACTIVE"] / 8 / sq["dur_ns"]
        res["waves"] = sq["SQ_WAVES"]
        res["rocprof_VGPR_Count"] = sq["vgpr"]   # rocprof's field (the code object says 128 VGPRs)
        res["scratch_bytes_per_lane"] = sq["scratch"]
    classes = os.path.join(out, "classes")
    rates = os.environ.get("RT_VALU_RATES", os.path.join(prof, "valu_rates.log"))
    if os.path.isdir(classes) and os.path.exists(rates):
        import valu_issue_model as vim
        os.makedirs(prof, exist_ok=True)
        model_path = os.path.join(prof, "valu_issue_model.json")
        clock = str(res.get("effective_clock_ghz", ""))   # the SQ pass's GRBM clock
        sys.argv = ["valu_issue_model.py", rates, classes, model_path, "", str(samples), config, clock]
        vim.main()
        with open(model_path) as f:
            m = json.load(f)
        res["valu_issue_cycles_per_sample"] = m["valu_issue_cycles_per_sample"]
        res["valu_issue_cycles_per_instr"] = m["valu_issue_cycles_per_launch"] / m["valu_insts_per_launch"]
        res["valu_issue_frac_weighted"] = m["valu_issue_frac_pmc_pass"]
        res["valu_issue_model"] = os.path.relpath(model_path, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    os.makedirs(prof, exist_ok=True)
    with open(os.path.join(prof, "traffic.json"), "w") as f:
        json.dump(res, f, indent=1)
    lines = ["# PMC summary (timed megakernel, separate rocprofv3 passes)", ""]
    lines += [f"- {k}: {v:.4g}" if isinstance(v, float) else f"- {k}: {v}" for k, v in res.items()]
    with open(os.path.join(prof, "pmc_summary.md"), "w") as f:
        f.write("\n".join(lines) + "\n")
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
