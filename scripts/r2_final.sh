#!/bin/bash
# Round-2 closing measurement: full GPU suite (verbose), default bench line (config 4 + CPU baseline),
# kernel trace/stats of config 4, PMC passes of the config-4 PC step
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v -s --timeout 300 --timeout-method thread > gpurun_out/gputest_final.log 2>&1 &&
timeout -k 10 600 python bench.py > gpurun_out/bench_final.json 2> gpurun_out/bench_final.err &&
rm -rf gpurun_out/prof_c4 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ode-calls 1 > gpurun_out/prof_c4.log 2>&1 &&
rm -rf gpurun_out/pmc_c4 &&
bash scripts/pmc_passes.sh gpurun_out/pmc_c4 256 > gpurun_out/pmc_c4.log 2>&1 &&
python scripts/pmc_pc_json.py gpurun_out/pmc_c4 12800 > gpurun_out/pmc_pc_step_config4.json
