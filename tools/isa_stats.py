#!/usr/bin/env python3
"""tools/isa_stats.py [--src DIR] [-DNAME=V ...] — static instruction statistics of the timed
megakernel variants (c4 / c3 / c2 symbols of tools/valu_issue_model.py) from the device
assembly: VALU / SALU / v_mov / v_readlane / LDS / global / scratch instruction counts,
and the resource usage (VGPRs, scratch bytes per lane).

--src DIR compiles DIR/csrc/hip/rt_kernel.hip (e.g. a `git worktree` of another revision)
instead of the tree's.  Used to check that a change meant to remove register moves does
not add spills (RT_SHADE_LEAN)."""
import collections
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = "peter-shirley-ray-tracing-the-next-week_amd"
VARIANTS = {
    "c4": "_ZN12_GLOBAL__N_113rt_megakernelILb0ELb0ELi2ELi16ELi1EEEv12RtKernelArgs",
    "c3": "_ZN12_GLOBAL__N_113rt_megakernelILb0ELb0ELi2ELi12ELi1EEEv12RtKernelArgs",
    "c2": "_ZN12_GLOBAL__N_113rt_megakernelILb0ELb0ELi2ELi1ELi2EEEv12RtKernelArgs",
}


def build_asm(src_root, defs):
    out = os.path.join(tempfile.mkdtemp(), "rt_kernel.s")
    pkg = os.path.join(src_root, PKG)
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "-ffp-contract=off",
           "-I" + os.path.join(src_root, "include"), "-I" + os.path.join(pkg, "csrc"),
           "-I" + os.path.join(pkg, "csrc", "host"), "-I" + os.path.join(pkg, "csrc", "hip"),
           "--offload-arch=gfx950", "-munsafe-fp-atomics", "-cuid=rt_kernel", "--cuda-device-only", "-S",
           os.path.join(pkg, "csrc", "hip", "rt_kernel.hip"), "-o", out] + defs
    subprocess.run(cmd, check=True, capture_output=True)
    return out


def stats(asm, symbol):
    c = collections.Counter()
    inside = False
    meta = {}
    for line in open(asm):
        if line.startswith(symbol + ":"):
            inside = True
            continue
        if inside and line.startswith("\t.section") or (inside and line.startswith(".Lfunc_end")):
            inside = False
        if inside:
            m = re.match(r"\s+([vsgdb][a-z0-9_]+)", line)
            if not m:
                continue
            op = m.group(1)
            if op.startswith("v_"):
                c["valu"] += 1
                if op.startswith("v_mov") or op.startswith("v_pk_mov"):
                    c["v_mov"] += 1
                if op.startswith("v_readlane") or op.startswith("v_writelane"):
                    c["v_read/writelane"] += 1
                if op.startswith("v_cndmask"):
                    c["v_cndmask"] += 1
            elif op.startswith("s_"):
                c["salu/smem/branch"] += 1
            elif op.startswith("ds_"):
                c["lds"] += 1
            elif op.startswith("global_") or op.startswith("buffer_") or op.startswith("flat_"):
                c["vmem"] += 1
            elif op.startswith("scratch_"):
                c["scratch"] += 1
        m = re.match(r"\s+\.(vgpr_count|sgpr_count|private_segment_fixed_size):\s+(\d+)", line)
        if m and symbol in meta.get("_cur", ""):
            meta[m.group(1)] = int(m.group(2))
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            meta["_cur"] = m.group(1)
    return c


def main():
    args = sys.argv[1:]
    src = ROOT
    if "--src" in args:
        i = args.index("--src")
        src = args[i + 1]
        del args[i:i + 2]
    asm = build_asm(src, args)
    text = open(asm).read()
    for cfg, sym in VARIANTS.items():
        c = stats(asm, sym)
        m = re.search(r"\.name:\s+" + re.escape(sym) + r"(.*?)\.vgpr_count:\s+(\d+)", text, re.S)
        scr = re.search(re.escape(sym) + r"\.private_seg_size, (\d+)", text)
        print(f"{cfg}: " + " ".join(f"{k} {v}" for k, v in sorted(c.items())) +
              (f" | scratch/lane {scr.group(1)}" if scr else ""))


if __name__ == "__main__":
    main()
