"""Concurrency of two kernel families in a rocprofv3 kernel trace (CSV).

    python3 tools/overlap.py <kernel_trace.csv | dir> --a 'rccl|nccl' --b 'cnn_bwd'

For every dispatch of family A (regex on the kernel name) it reports how much of its
[start, end) interval overlaps dispatches of family B, e.g. whether the fc bucket's RCCL
all-reduce runs beside the conv backward (the rccl-early step structure)."""
from __future__ import annotations

import argparse
import csv
import glob
import os
import re


def load(path):
    files = glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True) \
        if os.path.isdir(path) else [path]
    rows = []
    for f in files:
        for r in csv.DictReader(open(f)):
            rows.append((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    return sorted(rows, key=lambda t: t[1])


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--a", default="rccl|nccl|Nccl|Rccl")
    ap.add_argument("--b", default="cnn_bwd")
    a = ap.parse_args()
    rows = load(a.trace)
    fa = [r for r in rows if re.search(a.a, r[0])]
    fb = [r for r in rows if re.search(a.b, r[0])]
    if not fa or not fb:
        print(f"no dispatches: {len(fa)} of A ({a.a}), {len(fb)} of B ({a.b})")
        return
    tot, ov, hit = 0, 0, 0
    for name, s, e in fa:
        o = sum(max(0, min(e, be) - max(s, bs)) for _, bs, be in fb if bs < e and be > s)
        tot += e - s
        ov += o
        hit += o > 0
    print(f"A = {a.a}: {len(fa)} dispatches, {tot / len(fa) / 1e3:.2f} us mean")
    print(f"B = {a.b}: {len(fb)} dispatches, "
          f"{sum(e - s for _, s, e in fb) / len(fb) / 1e3:.2f} us mean")
    print(f"A dispatches overlapping B: {hit} of {len(fa)}; "
          f"overlapped time {ov / 1e3:.1f} of {tot / 1e3:.1f} us ({100 * ov / max(1, tot):.0f} %)")
    names = sorted({n[:60] for n, _, _ in fa})
    print("A kernels: " + "; ".join(names[:4]))


if __name__ == "__main__":
    main()
