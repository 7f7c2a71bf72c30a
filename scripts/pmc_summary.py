"""Summarise rocprofv3 --pmc CSVs: mean counter value per dispatch, per kernel.
usage: python scripts/pmc_summary.py DIR [kernel-substring ...]"""
import collections
import csv
import glob
import json
import sys

d = sys.argv[1]
subs = sys.argv[2:]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    rows = list(csv.DictReader(open(f)))
    per = collections.defaultdict(float)
    names = {}
    for r in rows:
        key = (r["Dispatch_Id"], r["Counter_Name"])
        per[key] += float(r["Counter_Value"])
        names[r["Dispatch_Id"]] = r["Kernel_Name"]
    for (disp, cname), v in per.items():
        acc[names[disp]][cname].append(v)
out = {}
for k, cs in acc.items():
    if subs and not any(s in k for s in subs):
        continue
    out[k[:70]] = {c: (sum(v) / len(v), len(v)) for c, v in sorted(cs.items())}
print(json.dumps(out, indent=1))
