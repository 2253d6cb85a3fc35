"""Condense an A/B run (tools/gpu_env_ab.sh, tools/gpu_ab_b.sh): bench img/s per variant and
the in-step per-kernel means from the summarised traces.

    python tools/ab_report.py gpurun_out/env_ab.log gpurun_out/env_prof
"""
import glob
import json
import os
import sys


def main():
    log, prof = sys.argv[1], sys.argv[2]
    head = None
    for line in open(log):
        if line.startswith("=="):
            head = line.strip("= \n")
        elif line.startswith("{"):
            d = json.loads(line)
            print(f"{head:50s} {d['value']:>12,.0f} img/s  {d['ms_per_step'] * 1e3:7.2f} us/step")
    for f in sorted(glob.glob(os.path.join(prof, "*.md"))):
        ks = []
        for line in open(f):
            p = [x.strip() for x in line.split("|")]
            if len(p) > 5 and p[2].isdigit() and int(p[2]) >= 150:
                ks.append(f"{p[1].split('<')[0].replace('_kernel', '')} {p[4]}")
        print(os.path.basename(f)[:-3].ljust(40), "; ".join(ks))


if __name__ == "__main__":
    main()
