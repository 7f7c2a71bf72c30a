#!/bin/bash
# Energy encoder beside vs after the score sampler (config 4), each with a kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for ov in 1 0; do
  timeout -k 10 300 python bench.py --no-cpu-baseline --ode-calls 0 --energy-overlap $ov > gpurun_out/bench_ov$ov.json 2> gpurun_out/bench_ov$ov.err || exit 1
done
rm -rf gpurun_out/prof_ov0 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ov0 -o ov0 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ode-calls 0 --energy-overlap 0 > gpurun_out/prof_ov0.log 2>&1
