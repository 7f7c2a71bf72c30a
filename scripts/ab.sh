#!/bin/bash
# Same-box A/B of library variants: alternates kbench runs (ABAB...) so clock drift between boxes
# does not decide the comparison.  usage: scripts/ab.sh {--pc|--enc} ROUNDS LIB1 LIB2 ...
MODE=$1; ROUNDS=$2; shift 2
for r in $(seq 1 "$ROUNDS"); do
  for L in "$@"; do
    GENPOSE_HIP_LIB=$L timeout -k 10 200 python scripts/kbench.py "$MODE" > gpurun_out/ab.json 2>&1 || exit 1
    echo "$r $L $(python -c "import json,re;t=open('gpurun_out/ab.json').read();d=json.loads(t[t.index('{'):]);print(' '.join(f'{k}={v.get(\"us_per_launch\",v.get(\"ms\")):.2f}' for k,v in d.items() if 'score' not in k))")"
  done
done
