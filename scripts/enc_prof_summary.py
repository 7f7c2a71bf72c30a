"""Per-launch durations of one steady-state encoder pass from gpurun_out/prof_enc (enc_prof.sh)."""
import csv
import sys

path = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/prof_enc/enc_kernel_trace.csv"
rows = list(csv.DictReader(open(path)))
seq = [(r["Kernel_Name"][:44], int(r["Grid_Size_X"]), int(r["Grid_Size_Y"]), int(r["Grid_Size_Z"]),
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1000) for r in rows]
idx = [i for i, x in enumerate(seq) if "fps" in x[0]]
i0, i1 = idx[1], idx[2]
tot = 0.0
for x in seq[i0:i1]:
    print(f"{x[0]:46s} grid=({x[1]},{x[2]},{x[3]}) {x[4]:9.1f} us")
    tot += x[4]
print(f"total {tot:.1f} us (kernel time, one B=64 pass)")
