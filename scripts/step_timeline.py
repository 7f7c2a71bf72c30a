"""One config-4 bench step's timeline from a rocprofv3 kernel trace: every launch that is not a PC step,
with its stream, and the span of the PC-step run, for the last timed step."""
import csv
import sys

r = [x for x in csv.DictReader(open(sys.argv[1])) if 'copyBuffer' not in x['Kernel_Name']]
r.sort(key=lambda x: int(x['Start_Timestamp']))
fps = [i for i, x in enumerate(r) if 'fps_chain' in x['Kernel_Name']]
i0 = fps[-2]   # the last step's first encoder (two encoders per step)
t0 = int(r[i0]['Start_Timestamp'])
pc = [x for x in r[i0:] if 'pc_step' in x['Kernel_Name']]
end = int(pc[-1]['End_Timestamp']) if pc else int(r[-1]['End_Timestamp'])
for x in r[i0:]:
    s, e = int(x['Start_Timestamp']), int(x['End_Timestamp'])
    if s > end + 2_000_000:
        break
    if 'pc_step' in x['Kernel_Name']:
        continue
    print(f"{(s - t0) / 1e3:9.1f} {(e - s) / 1e3:8.1f} q{x['Queue_Id']:>3} {x['Kernel_Name'][:60]}")
if pc:
    print(f"pc_step: {len(pc)} launches from {(int(pc[0]['Start_Timestamp']) - t0) / 1e3:.1f} to {(end - t0) / 1e3:.1f} us")
