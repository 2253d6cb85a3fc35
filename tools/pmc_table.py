"""Per-kernel PMC table with derived values, readable without the CSVs.

    python3 tools/pmc_table.py --title T --trace <kernel_trace.csv> <pass dirs or CSVs...>

Inputs: the ``*counter_collection.csv`` of each rocprofv3 ``--pmc`` pass (one pass per
counter group, tools/pmc_run.sh) and the ``*kernel_trace.csv`` of a ``--kernel-trace`` run of
the same program (kernel durations).  Every value is the mean over the kernel's dispatches.

Derived columns (units and sources; MI355X_MICROARCH.md, "rocprofv3 PMC slots", "DVFS"):
  dur us        kernel-trace End - Start (back-to-back dispatches: includes the launch gap)
  waves/CU      SQ_WAVES / 256 CUs
  MFMA busy %   SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x dur x 2.4 GHz): the share of the
                dispatch's SIMD-cycles the matrix cores were busy, at the peak clock (a lower
                bound when the chip runs slower).  GRBM_GUI_ACTIVE / 8 / dur reads 3-6 GHz on
                these microsecond dispatches (MI355X_MICROARCH.md: it reads high below
                ~0.3 ms), so it is not used as the clock
  VALU/wave     SQ_INSTS_VALU / SQ_WAVES (wave64 vector instructions, MFMA included)
  LDS confl %   SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE (extra cycles over LDS-active cycles)
  wait %        SQ_WAIT_ANY / SQ_WAVE_CYCLES (waves parked on s_waitcnt / barriers)
  issue-stall % SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES
  rd MB, wr MB  FETCH_SIZE, WRITE_SIZE (KiB) -> MB.  gfx950 FETCH_SIZE counts wide streaming
                reads at half their bytes; it is reported as measured (a lower bound)
  GB/s          (rd + wr) / dur
  L2 hit %      TCC_HIT_sum / (TCC_HIT_sum + TCC_MISS_sum)
"""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re
from collections import defaultdict

NAMES = ("cnn", "fc1", "conv", "optim", "lin", "f32", "gather", "xgmi")


def short(n: str) -> str:
    n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", n)      # anonymous-namespace mangling
    m = re.search(r"(\w+_kernel)(?:I(\w))?", n)
    if not m:
        return n[:40]
    return m.group(1)


def csvs(paths, pattern):
    out = []
    for p in paths:
        if os.path.isdir(p):
            out += glob.glob(os.path.join(p, "**", pattern), recursive=True)
        elif p.endswith(".csv"):
            out.append(p)
    return out


def load_counters(files):
    vals = defaultdict(lambda: defaultdict(list))
    for path in files:
        for r in csv.DictReader(open(path)):
            vals[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in vals.items()}


def load_durations(files):
    dur = defaultdict(list)
    for path in files:
        for r in csv.DictReader(open(path)):
            dur[short(r["Kernel_Name"])].append(
                (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: (sorted(v)[len(v) // 2], len(v)) for k, v in dur.items()}


def table(counters, durations, title=""):
    hdr = ["kernel", "dur us", "waves/CU", "MFMA busy %", "VALU/wave",
           "LDS confl %", "wait %", "issue-stall %", "rd MB", "wr MB", "GB/s", "L2 hit %"]
    rows = [f"### {title}" if title else "", "", "| " + " | ".join(hdr) + " |",
            "|---|" + "---:|" * (len(hdr) - 1)]
    nan = float("nan")
    for k in sorted(counters, key=lambda k: -durations.get(k, (0, 0))[0]):
        if not any(s in k for s in NAMES):
            continue
        d = counters[k]
        f = lambda c: d.get(c, nan)
        us = durations.get(k, (nan, 0))[0]
        waves = f("SQ_WAVES")
        rd = f("FETCH_SIZE") * 1024 / 1e6
        wr = f("WRITE_SIZE") * 1024 / 1e6
        hit, miss = f("TCC_HIT_sum"), f("TCC_MISS_sum")
        cells = [k, f"{us:.2f}", f"{waves / 256:.1f}",
                 f"{100 * f('SQ_VALU_MFMA_BUSY_CYCLES') / (1024 * us * 2.4e3):.1f}",
                 f"{f('SQ_INSTS_VALU') / waves:.0f}",
                 f"{100 * f('SQ_LDS_BANK_CONFLICT') / f('SQ_LDS_IDX_ACTIVE'):.1f}"
                 if f("SQ_LDS_IDX_ACTIVE") > 0 else "-",
                 f"{100 * f('SQ_WAIT_ANY') / f('SQ_WAVE_CYCLES'):.0f}",
                 f"{100 * f('SQ_WAIT_INST_ANY') / f('SQ_WAVE_CYCLES'):.0f}",
                 f"{rd:.2f}", f"{wr:.2f}", f"{(rd + wr) * 1e3 / us:.0f}",
                 f"{100 * hit / (hit + miss):.0f}"]
        rows.append("| " + " | ".join(c.replace("nan", "-") for c in cells) + " |")
    return "\n".join(rows)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--title", default="")
    ap.add_argument("--trace", action="append", default=[])
    ap.add_argument("paths", nargs="+")
    a = ap.parse_args()
    counters = load_counters(csvs(a.paths, "*counter_collection.csv"))
    durations = load_durations(csvs(a.trace, "*kernel_trace.csv"))
    print(table(counters, durations, a.title))


if __name__ == "__main__":
    main()
