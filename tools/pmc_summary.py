"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel (short names)."""
import csv
import re
import sys
from collections import defaultdict


def short(n):
    m = re.search(r"(\w+_kernel)", n)
    return (m.group(1) if m else n)[:28]


def load(path):
    vals = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(path)):
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return vals


if __name__ == "__main__":
    for path in sys.argv[1:]:
        vals = load(path)
        ctrs = sorted({c for d in vals.values() for c in d})
        print(path)
        print(f"{'kernel':28s} " + " ".join(f"{c[3:][:14]:>14s}" for c in ctrs))
        for k, d in vals.items():
            if not any(s in k for s in ("cnn", "fc1", "conv", "optim", "lin")):
                continue
            print(f"{k:28s} " + " ".join(f"{sum(d[c]) / max(1, len(d[c])):14.0f}" for c in ctrs))
