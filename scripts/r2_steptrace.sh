#!/bin/bash
# Kernel trace of config-4 bench steps (one step's non-sampler timeline is read from it)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/prof_step &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step -o st -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline --ode-calls 1 > gpurun_out/prof_step.log 2>&1
