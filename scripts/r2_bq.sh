#!/bin/bash
# Ball query with two centroids per wave + level-0 xyz projection: GPU suite, ball-query microbench,
# encoder timing + kernel trace, config-4 bench
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 100 python scripts/bq_bench.py > gpurun_out/bq.json 2> gpurun_out/bq.err &&
timeout -k 10 200 python scripts/enc_bench.py 256 10 > gpurun_out/enc_main.json 2> gpurun_out/enc_main.err &&
rm -rf gpurun_out/prof_enc &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enc -o enc -- python3 scripts/enc_bench.py 256 3 > gpurun_out/prof_enc.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench.json 2> gpurun_out/bench.err
