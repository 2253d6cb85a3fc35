"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel (short names)."""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    n = re.sub(r"^_ZN12_GLOBAL__N_1\d+", "", n)      # anonymous-namespace mangling
    m = re.search(r"(\w+_kernel)", n)
    return (m.group(1) if m else n)[:28]


def load(path):
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


def table(paths):
    """One markdown row per kernel from every pass (counters merged by kernel name)."""
    allv = defaultdict(dict)
    for path in paths:
        for k, d in load(path).items():
            for c, v in d.items():
                allv[k][c] = sum(v) / max(1, len(v))
    rows = []
    hdr = ("| kernel | waves | wave life (cyc) | VALU / wave | MFMA / wave | LDS / wave | "
           "stall % | MFMA busy / SIMD (cyc) | LDS confl % | FETCH KB | WRITE KB |")
    rows.append(hdr)
    rows.append("|---|" + "---:|" * (hdr.count("|") - 2))
    for k, d in allv.items():
        if not any(s in k for s in ("cnn", "fc1", "conv", "optim", "lin")):
            continue
        w = d.get("SQ_WAVES", 0) or 1
        life = d.get("SQ_WAVE_CYCLES", 0) / w * 4          # SQ_WAVE_CYCLES counts quad-cycles
        f = lambda c: d.get(c, float("nan"))
        stall = 100 * f("SQ_WAIT_INST_ANY") / max(1, f("SQ_WAVE_CYCLES"))
        confl = 100 * f("SQ_LDS_BANK_CONFLICT") / max(1, f("SQ_LDS_IDX_ACTIVE"))
        rows.append(f"| {k} | {w:.0f} | {life:.0f} | {f('SQ_INSTS_VALU') / w:.0f} | "
                    f"{f('SQ_INSTS_MFMA') / w:.0f} | {f('SQ_INSTS_LDS') / w:.0f} | {stall:.0f} | "
                    f"{f('SQ_VALU_MFMA_BUSY_CYCLES') / 1024:.0f} | {confl:.0f} | "
                    f"{f('FETCH_SIZE'):.0f} | {f('WRITE_SIZE'):.0f} |")
    return "\n".join(rows)


if __name__ == "__main__":
    if sys.argv[1:2] == ["--table"]:
        print(table(sys.argv[2:]))
        sys.exit(0)
    for path in sys.argv[1:]:
        vals = load(path)
        ctrs = sorted({c for d in vals.values() for c in d})
        print(path)
        print(f"{'kernel':28s} " + " ".join(f"{c[3:][:14]:>14s}" for c in ctrs))
        for k, d in vals.items():
            if not any(s in k for s in ("cnn", "fc1", "conv", "optim", "lin")):
                continue
            print(f"{k:28s} " + " ".join(f"{sum(d[c]) / max(1, len(d[c])):14.0f}" for c in ctrs))
