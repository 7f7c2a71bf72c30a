#!/bin/bash
# Energy encoder placement A/B at config 4: after the sampler (0), beside the score encoder (2)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ov in 0 2; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --ode-calls 0 --energy-overlap $ov > gpurun_out/bench_ov$ov.json 2> gpurun_out/bench_ov$ov.err || exit 1
done
