#!/bin/bash
# Same-box A/B of an environment setting on the full bench step, alternating ABAB...
# usage: bash scripts/ab_env.sh TAG ROUNDS "BENCH ARGS" VAR VALUE1 VALUE2 ...
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
TAG=$1; ROUNDS=$2; ARGS=$3; VAR=$4; shift 4
for r in $(seq 1 "$ROUNDS"); do
  for V in "$@"; do
    env "$VAR=$V" timeout -k 10 300 python bench.py $ARGS > gpurun_out/${TAG}.json 2> gpurun_out/${TAG}.err || exit 1
    echo "$r $VAR=$V $(python -c "import json;d=json.loads(open('gpurun_out/${TAG}.json').read().strip().splitlines()[-1]);r=d['roofline'];print(f\"ms_per_step={d['ms_per_step']:.3f} sampler_ms={r.get('sampler_ms_per_step',0):.3f} pc_us={r['avg_launch_us']:.2f}\")")"
  done
done
