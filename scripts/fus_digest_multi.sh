#!/bin/bash
# Multi-process determinism check of the DINO-pointwise fused encoder: PROCS processes on cuda:0 each run
# scripts/fus_digest.py REPS times at once; every output digest must be the same.
# usage: bash scripts/fus_digest_multi.sh PROCS REPS OUT
P=${1:-6}; R=${2:-3}; OUT=${3:-gpurun_out/fus_multi.jsonl}
: > "$OUT"
pids=()
for i in $(seq 1 "$P"); do
  ( for r in $(seq 1 "$R"); do timeout -k 10 300 python scripts/fus_digest.py 256 || exit 1; done ) >> "$OUT" 2>/dev/null &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait "$p" || rc=1; done
python - "$OUT" <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")]
print(json.dumps({"runs": len(d), "digests": sorted({x["digest"] for x in d})}))
PY
exit $rc
