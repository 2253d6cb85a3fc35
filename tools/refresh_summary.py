"""Condense a refresh bench log (tools/gpu_refresh.sh: '## <command>' lines, each followed by
bench.py's JSON line) into a markdown table.

    python tools/refresh_summary.py profiles/r4/final/bench.jsonl
"""
import json
import sys


def structure(d):
    comm = d.get("comm") or {}
    parts = [comm.get("data_plane", "")]
    for k in ("transport", "chosen", "rccl_mode"):
        if comm.get(k):
            parts.append(str(comm[k]))
    knobs = d.get("knobs") or {}
    parts += [f"{k}={v}" for k, v in knobs.items()]
    return " ".join(p for p in parts if p)


def main(path):
    rows, cmd = [], None
    for line in open(path):
        line = line.strip()
        if line.startswith("## "):
            cmd = line[3:]
        elif line.startswith("{"):
            d = json.loads(line)
            cfg = d.get("config", {})
            rows.append((cmd, d["value"], d["ms_per_step"] * 1000, d.get("n_gpus"),
                         cfg.get("global_batch"), d.get("dtype"), structure(d)))
    print("| command | img/s | µs/step | N | global batch | dtype | structure |")
    print("|---|---:|---:|---:|---:|---|---|")
    for r in rows:
        print(f"| `{r[0]}` | {r[1]:,.0f} | {r[2]:.1f} | {r[3]} | {r[4]} | {r[5]} | {r[6]} |")


if __name__ == "__main__":
    main(sys.argv[1])
