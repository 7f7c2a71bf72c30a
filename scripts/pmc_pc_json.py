"""pc_step_kernel HBM traffic per launch from the PMC passes of scripts/pmc_passes.sh:
FETCH_SIZE x2 (gfx950 reports half the bytes of 16-B/lane streaming reads, MI355X_MICROARCH.md
§HBM) + WRITE_SIZE, both in KB (1024 B); L2 hit rate and mean L2 read latency alongside.
usage: python scripts/pmc_pc_json.py PMC_DIR ROWS > profiles/rN/pmc_pc_step_configX.json"""
import collections
import csv
import glob
import json
import sys

d, rows = sys.argv[1], int(sys.argv[2])
acc = collections.defaultdict(list)
name = None
for f in glob.glob(f"{d}/**/*counter_collection.csv", recursive=True):
    per = collections.defaultdict(float)
    for r in csv.DictReader(open(f)):
        if "pc_step_kernel" not in r["Kernel_Name"]:
            continue
        name = r["Kernel_Name"]
        per[(r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
    for (_, c), v in per.items():
        acc[c].append(v)
m = {c: sum(v) / len(v) for c, v in acc.items()}
n = len(acc.get("FETCH_SIZE", []))
out = {"kernel": name, "rows": rows,
       "source": f"rocprofv3 --pmc, one counter group per pass (scripts/pmc_passes.sh), mean over {n} dispatches "
                 f"of scripts/pmc_target.py",
       "correction": "FETCH_SIZE x2 (gfx950), WRITE_SIZE as is; KB=1024 B",
       "fetch_size_kb": m.get("FETCH_SIZE"), "write_size_kb": m.get("WRITE_SIZE"),
       "hbm_bytes_per_launch": (2 * m["FETCH_SIZE"] + m["WRITE_SIZE"]) * 1024,
       "algorithmic_bytes_per_launch": rows * 72,
       "note": "fabric reads are dominated by each XCD's L2 re-fetching the streamed head weights (1.57 MB of f16x3 planes) once "
               "per launch (the kernel boundary invalidates L2); served from the 256 MB Infinity Cache"}
if "SQ_VALU_MFMA_BUSY_CYCLES" in m:
    # summed over every SIMD of the chip; the launch occupies ceil(rows / tile) CUs (one workgroup each)
    tile = 64 if rows > 8192 else (32 if rows > 4096 else 16)
    simds = 4 * min(256, -(-rows // tile))
    out["mfma_busy_cycles_per_active_simd"] = m["SQ_VALU_MFMA_BUSY_CYCLES"] / simds
    out["grbm_gui_active_per_xcd"] = m.get("GRBM_GUI_ACTIVE", 0) / 8
    out["pmc_note"] = ("counters under --pmc stretch the launch (GRBM_GUI_ACTIVE per XCD is the profiled duration); "
                       "divide the MFMA busy cycles by the un-profiled workgroup lifetime (scripts/pc_trace.py) for "
                       "the MFMA utilisation")
if "SQ_INSTS_VALU" in m:
    out["valu_insts"] = m["SQ_INSTS_VALU"]
    out["lds_bank_conflict_cycles"] = m.get("SQ_LDS_BANK_CONFLICT")
if "TCC_HIT_sum" in m:
    out["tcc_hit_rate"] = m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"])
if "TCP_TCC_READ_REQ_sum" in m:
    out["avg_l2_read_latency_cycles"] = m["TCP_TCC_READ_REQ_LATENCY_sum"] / m["TCP_TCC_READ_REQ_sum"]
print(json.dumps(out, indent=1))
