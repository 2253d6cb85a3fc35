"""Per-step kernel timeline from a rocprofv3 --kernel-trace --output-format csv run.

    python tools/step_timeline.py <run_kernel_trace.csv> [--anchor cnn_fwd] [--last N]

Prints, for the last N steps (a step starts at each `anchor` kernel), every
kernel's start/end offset in us relative to the step start, so overlap between
the compute stream and the communication stream (xgmi_allreduce / RCCL) is
visible, plus the mean duration and mean start offset of each kernel.
"""
import argparse
import csv
from collections import defaultdict


def short(name):
    for pre in ("void ", "(anonymous namespace)::", "_ZN12_GLOBAL__N_1"):
        name = name.replace(pre, "")
    name = name.split("(")[0].split("<")[0].lstrip("0123456789")
    return name[:40]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--anchor", default="cnn_fwd")
    ap.add_argument("--last", type=int, default=3)
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.csv)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]),
                  r["Queue_Id"]) for r in rows))
    starts = [i for i, k in enumerate(ks) if a.anchor in k[2]]
    steps = []
    for j in range(len(starts) - 1):
        steps.append(ks[starts[j]:starts[j + 1]])
    steps = steps[-max(a.last, 20):]
    for st in steps[-a.last:]:
        t0 = st[0][0]
        print(f"-- step ({(st[-1][1] - t0) / 1e3:.1f} us to last end)")
        for s, e, n, q in st:
            print(f"   q{q:>2} {n:40s} {(s - t0) / 1e3:8.2f} -> {(e - t0) / 1e3:8.2f}  ({(e - s) / 1e3:6.2f})")
    agg = defaultdict(lambda: [0, 0.0, 0.0])
    for st in steps:
        t0 = st[0][0]
        for s, e, n, q in st:
            g = agg[n]
            g[0] += 1
            g[1] += (e - s) / 1e3
            g[2] += (s - t0) / 1e3
    print(f"-- mean over {len(steps)} steps: kernel, calls/step, dur us, start us")
    for n, (c, d, s) in sorted(agg.items(), key=lambda kv: kv[1][2] / kv[1][0]):
        print(f"   {n:40s} {c / len(steps):5.2f} {d / c:8.2f} {s / c:8.2f}")
    per = [(st[-1][0] - st[0][0]) for st in steps]
    gaps = [(steps[i + 1][0][0] - steps[i][0][0]) / 1e3 for i in range(len(steps) - 1)]
    if gaps:
        print(f"-- mean step period {sum(gaps) / len(gaps):.2f} us")


if __name__ == "__main__":
    main()
