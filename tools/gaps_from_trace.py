"""Idle gaps inside the windows of tools/graph_gaps.py, from its rocprofv3 kernel trace: the
windows start after the marker spin kernels (torch.cuda._sleep) (one per window, in the order the tool runs them).

    python tools/gaps_from_trace.py run_results.db NAMES_IN_ORDER...
"""
import collections
import sqlite3
import statistics
import sys

from rocpd_summary import short

db, names = sys.argv[1], sys.argv[2:]
rows = [(short(n), s, e) for n, s, e in sqlite3.connect(db).execute(
    "select name, start, end from kernels order by start").fetchall()]
marks = [i for i, r in enumerate(rows) if "spin" in r[0]]
per = collections.defaultdict(list)
detail = collections.defaultdict(collections.Counter)
for w, i in enumerate(marks):
    name = names[w % len(names)]
    j = marks[w + 1] if w + 1 < len(marks) else len(rows)
    win = rows[i + 1:j]
    # the window's 20 steps: up to the 20th optimizer launch
    nopt, end = 0, len(win)
    for k, r in enumerate(win):
        if r[0].startswith("optim"):
            nopt += 1
            if nopt == 20:
                end = k + 1
                break
    win = win[:end]
    idle, last = 0.0, win[0][2]
    for a, b in zip(win, win[1:]):
        g = max(0.0, (b[1] - max(last, a[2])) / 1e3)
        last = max(last, b[2])
        idle += g
        if g > 3.0:
            detail[name][f"{a[0][:24]} -> {b[0][:24]}"] += 1
    span = (win[-1][2] - win[0][1]) / 1e3
    per[name].append((span, idle))
for n in names:
    if per[n]:
        print(f"{n:9s} span {statistics.median(s for s, _ in per[n]):7.1f} us, idle "
              f"{statistics.median(i for _, i in per[n]):6.1f} us  gaps>3us: "
              + "; ".join(f"{k} x{v}" for k, v in detail[n].most_common(6)))
