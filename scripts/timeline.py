"""Idle gaps on the GPU timeline of a kernel trace (rocprofv3 --kernel-trace csv): per step of
bench.py, kernel busy time vs wall span, and the largest gaps with the kernels around them."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_bench/bench_kernel_trace.csv"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:40]) for r in rows]
# steps start at each fps_chain launch
starts = [i for i, e in enumerate(ev) if "fps_chain" in e[2]]
for si in range(len(starts) - 1):
    seg = ev[starts[si]:starts[si + 1]]
    busy, t_end, gaps = 0, seg[0][0], []
    for s, e, n in seg:
        if s > t_end:
            gaps.append((s - t_end, n))
        busy += max(0, e - max(s, t_end))
        t_end = max(t_end, e)
    span = t_end - seg[0][0]
    gaps.sort(reverse=True)
    print(f"step {si}: span {span/1e6:.3f} ms busy {busy/1e6:.3f} ms idle {(span-busy)/1e6:.3f} ms; "
          f"largest gaps: " + ", ".join(f"{g/1e3:.1f}us before {n}" for g, n in gaps[:5]))
