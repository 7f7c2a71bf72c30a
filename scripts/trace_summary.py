"""Summarise a rocprofv3 kernel trace (CSV): per-kernel launch-time distribution, and for the PC
step kernel the per-call sum and the launches stalled behind side-stream work (> 2x median)."""
import csv
import json
import sys

import numpy as np


def main(path, calls_len=501):
    rows = list(csv.DictReader(open(path)))
    by = {}
    for r in rows:
        by.setdefault(r["Kernel_Name"].split("(")[0], []).append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    out = {"kernels": {}}
    for k, v in sorted(by.items(), key=lambda kv: -sum(kv[1])):
        d = np.array(v)
        out["kernels"][k] = {"calls": len(d), "total_ms": d.sum() / 1e6, "median_us": float(np.median(d)) / 1e3,
                             "p99_us": float(np.percentile(d, 99)) / 1e3, "max_us": d.max() / 1e3}
    pc = [v for k, v in by.items() if k.startswith("void pc_step_kernel")]
    if pc:
        d = np.array(pc[0])
        med = float(np.median(d))
        per = []
        for c in range(len(d) // calls_len):
            s = d[c * calls_len:(c + 1) * calls_len]
            st = s[s > 2 * med]
            per.append({"sum_ms": s.sum() / 1e6, "median_us": float(np.median(s)) / 1e3,
                        "stalled_launches": int(len(st)), "stalled_ms": st.sum() / 1e6})
        out["pc_step_calls"] = per
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 501)
