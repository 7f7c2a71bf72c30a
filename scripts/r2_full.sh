#!/bin/bash
# Round-2 re-entry: full GPU suite, default bench line (config 4, CPU baseline), kernel stats of config 4
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 500 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err &&
rm -rf gpurun_out/prof_c4 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ode-calls 1 > gpurun_out/prof_c4.log 2>&1
