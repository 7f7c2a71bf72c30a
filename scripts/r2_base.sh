#!/bin/bash
# Round-2 baseline: GPU tests, config-4 bench line, kernel trace of config 4 (timeline of the stalls)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --config 4 --no-cpu-baseline > gpurun_out/bench_c4.json 2> gpurun_out/bench_c4.err &&
rm -rf gpurun_out/prof_c4 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/prof_c4.log 2>&1
