"""Print a stretch of a rocprofv3 kernel trace as a timeline: every dispatch (all queues) with
its start relative to the first one shown, its duration, and the idle gap since the latest end
of anything before it -- what a per-kernel summary cannot show (overlap of the persistent
collective with the step, waits between launches).

    python tools/rocpd_timeline.py run_results.db [--after NAME --skip K] [--count N]

--after NAME / --skip K: start at the K-th dispatch of kernel NAME (default: the 100th
dispatch overall; launches over 200 us, the persistent collective, do not count as busy, past the warm-up and calibration).
"""
import argparse
import sqlite3

from rocpd_summary import short


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--after", default=None)
    ap.add_argument("--skip", type=int, default=100)
    ap.add_argument("--count", type=int, default=40)
    ap.add_argument("--title", default="kernel timeline")
    ap.add_argument("--last", type=int, default=None,
                    help="start N dispatches before the end of the trace (the timed window of a "
                         "short bench.py run sits near the end)")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = [(short(n), s, e) for n, s, e in
            c.execute("select name, start, end from kernels order by start").fetchall()]
    if a.last:
        i0 = max(0, len(rows) - a.last)
    elif a.after:
        hits = [i for i, r in enumerate(rows) if r[0].startswith(a.after)]
        i0 = hits[min(a.skip, len(hits) - 1)] if hits else 0
    else:
        i0 = min(a.skip, max(0, len(rows) - a.count))
    win = rows[i0:i0 + a.count]
    t0 = win[0][1]
    # long-lived launches (the persistent collective, > 200 us) do not count as busy: the idle
    # column is the compute chain's
    short_rows = [e for _, s, e in rows[:i0] if e - s < 200_000]
    last_end = max(short_rows) if short_rows else win[0][1]
    print(f"## {a.title}\n")
    print("| # | kernel | start us | dur us | idle before us |")
    print("|---:|---|---:|---:|---:|")
    for k, (n, s, e) in enumerate(win):
        idle = max(0.0, (s - last_end) / 1000.0)
        print(f"| {k} | {n} | {(s - t0) / 1000.0:.2f} | {(e - s) / 1000.0:.2f} | {idle:.2f} |")
        if e - s < 200_000:
            last_end = max(last_end, e)


if __name__ == "__main__":
    main()
