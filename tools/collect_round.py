#!/usr/bin/env python3
"""tools/collect_round.py OUT PROFILE_DIR — files a `tools/round_profile.sh` +
`tools/round_bench.sh` run (merged back into OUT, normally gpurun_out/) into
PROFILE_DIR (profiles/rNN/), the layout bench.py's roofline reads:

  PROFILE_DIR/{traffic.json,pmc_summary.md,valu_issue_model.json}   c4 (tools/pmc_traffic.py)
  PROFILE_DIR/<cfg>/...                                             c5, c5_nN, c3, c2
  PROFILE_DIR/pmc/<cfg>/pmc_{fetch,write,l2,sq,lds,lanes}.csv, classes/pmc_classes_{1,2}.csv
  PROFILE_DIR/lanes.json                                            tools/lanes_summary.py
  PROFILE_DIR/valu_rates.log                                        the issue-cost microbenchmark
  PROFILE_DIR/final/{bench_*.log,prof.log}, kernel_stats_c4.csv     tools/final_bench.sh
  PROFILE_DIR/wave_log_c4.json, stage_final.json                    tools/wave_log.py, tools/stage_profile.py

Run on the build host with the library the box ran (its kernel hash goes into the
summaries).  Missing inputs are skipped.
"""
import os
import shutil
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
# samples per launch of each profiled workload (bench.py CONFIGS; c5_nN: one rank's share)
SAMPLES = {"c4": 500 * 500 * 1000, "c5": 1000 * 1000 * 1000, "c3": 800 * 400 * 500, "c2": 400 * 400 * 200}


def samples_of(cfg):
    if cfg.startswith("c5_n"):
        return SAMPLES["c5"] // int(cfg[4:])
    return SAMPLES[cfg]


def cp(src, dst):
    if os.path.exists(src):
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copy(src, dst)
        return True
    return False


def main():
    out, prof = sys.argv[1], sys.argv[2]
    os.makedirs(prof, exist_ok=True)
    cp(os.path.join(out, "final_c4", "valu_rates.log"), os.path.join(prof, "valu_rates.log"))
    env = dict(os.environ, RT_VALU_RATES=os.path.join(prof, "valu_rates.log"))
    cfgs = sorted(d[len("final_"):] for d in os.listdir(out) if d.startswith("final_c") and
                  os.path.isdir(os.path.join(out, d)))
    for cfg in cfgs:
        src = os.path.join(out, "final_" + cfg)
        dst = prof if cfg == "c4" else os.path.join(prof, cfg)
        os.makedirs(dst, exist_ok=True)
        r = subprocess.run([sys.executable, os.path.join(HERE, "pmc_traffic.py"), src, dst, str(samples_of(cfg)), cfg],
                           env=env, stdout=subprocess.DEVNULL)
        if r.returncode == 3:   # counters of another build (pmc_traffic.py): left out
            print("profile", cfg, "skipped: another build's counters")
            continue
        r.check_returncode()
        pd = os.path.join(prof, "pmc", cfg)
        for k in ("fetch", "write", "l2", "sq", "lds"):
            cp(os.path.join(src, f"pmc_{k}", "run_counter_collection.csv"), os.path.join(pd, f"pmc_{k}.csv"))
        for i in (1, 2):
            cp(os.path.join(src, "classes", f"pass{i}", "run_counter_collection.csv"),
               os.path.join(pd, "classes", f"pmc_classes_{i}.csv"))
        cp(os.path.join(out, "lanes_" + cfg, "run_counter_collection.csv"), os.path.join(pd, "pmc_lanes.csv"))
        print("profile", cfg, "->", dst)
    subprocess.run([sys.executable, os.path.join(HERE, "lanes_summary.py"), out, os.path.join(prof, "lanes.json")],
                   check=True, stdout=subprocess.DEVNULL)
    fin = os.path.join(out, "final")
    if os.path.isdir(fin):
        for f in sorted(os.listdir(fin)):
            if f.endswith(".log"):
                cp(os.path.join(fin, f), os.path.join(prof, "final", f))
        cp(os.path.join(fin, "prof", "run_kernel_stats.csv"), os.path.join(prof, "kernel_stats_c4.csv"))
    cp(os.path.join(out, "wave_log_c4.json"), os.path.join(prof, "wave_log_c4.json"))
    cp(os.path.join(out, "stage_final.json"), os.path.join(prof, "stage_final.json"))


if __name__ == "__main__":
    main()
