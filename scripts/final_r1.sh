#!/bin/bash
# Round-end refresh: default bench line (config 2) + its rocprof kernel stats, config 4 line.
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err &&
timeout -k 10 300 python bench.py --config 4 > gpurun_out/bench_config4_final.log 2>&1 &&
timeout -k 10 300 bash scripts/bench_prof.sh
