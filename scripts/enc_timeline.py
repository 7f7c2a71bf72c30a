"""Print one Light-encoder forward's launch timeline from a rocprofv3 kernel trace (the second forward)."""
import csv
import sys

r = [x for x in csv.DictReader(open(sys.argv[1])) if 'copyBuffer' not in x['Kernel_Name']]
r.sort(key=lambda x: int(x['Start_Timestamp']))
idx = [i for i, x in enumerate(r) if 'fps_chain' in x['Kernel_Name']]
i0 = idx[1]
t0 = int(r[i0]['Start_Timestamp'])
for x in r[i0:idx[2] if len(idx) > 2 else i0 + 24]:
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} {x['Kernel_Name'][:64]:64s} "
          f"grid {x['Grid_Size_X']}x{x['Grid_Size_Y']}x{x['Grid_Size_Z']}")
