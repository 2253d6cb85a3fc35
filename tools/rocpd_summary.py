"""Summarise a rocprofv3 (ROCm 7 rocpd SQLite) kernel trace into a markdown table.

    python tools/rocpd_summary.py gpurun_out/prof/run_results.db [--title T] [--steps N]

Per kernel: calls, total / mean / min / max duration (us), share of GPU time, plus the
steady-state per-step time (sum of per-kernel means of the kernels called >= N times)
and the mean launch gap between consecutive kernels of the step.
"""
import argparse
import re
import sqlite3
import statistics


def short(name: str) -> str:
    n = name.replace("(anonymous namespace)::", "").replace("void ", "")
    if n.startswith("_ZN"):
        # mangled nested name: a run of <len><identifier> pieces after "_ZN"
        ids, i = [], 3
        while True:
            m = re.match(r"\d+", n[i:])
            if not m:
                break
            ln = int(m.group(0))
            i += len(m.group(0))
            ids.append(n[i:i + ln])
            i += ln
        n = next((x for x in ids if x.endswith("kernel")), ids[-1] if ids else n)
        return n[:60]
    return n.split("(")[0][:60]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--title", default="rocprofv3 kernel trace")
    ap.add_argument("--steps", type=int, default=100,
                    help="kernels called at least this often are treated as per-step kernels")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = c.execute("select name, start, end from kernels order by start").fetchall()
    per = {}
    for name, s, e in rows:
        per.setdefault(short(name), []).append((e - s) / 1000.0)
    total = sum(sum(v) for v in per.values())
    print(f"## {a.title}\n")
    print("| kernel | calls | total us | mean us | min us | max us | % GPU |")
    print("|---|---:|---:|---:|---:|---:|---:|")
    for k, v in sorted(per.items(), key=lambda kv: -sum(kv[1])):
        print(f"| {k} | {len(v)} | {sum(v):.1f} | {statistics.mean(v):.2f} | {min(v):.2f} | "
              f"{max(v):.2f} | {100 * sum(v) / total:.1f} |")
    # torch / runtime kernels (graph capture and upload fills, copies) are not step kernels,
    # however often they run
    step = {k: statistics.mean(v) for k, v in per.items()
            if len(v) >= a.steps and not k.startswith(("at::", "__amd"))}
    if step:
        print(f"\nper-step kernels (called >= {a.steps}x): sum of means = "
              f"{sum(step.values()):.1f} us")
        names = set(step)
        seq = [(short(n), s, e) for n, s, e in rows if short(n) in names]
        gaps = [(seq[i + 1][1] - seq[i][2]) / 1000.0 for i in range(len(seq) - 1)]
        gaps = [g for g in gaps if g < 50.0]     # drop host-side pauses (epoch boundaries)
        if gaps:
            print(f"median gap between consecutive per-step kernels: "
                  f"{statistics.median(gaps):.2f} us over {len(gaps)} gaps")


if __name__ == "__main__":
    main()
