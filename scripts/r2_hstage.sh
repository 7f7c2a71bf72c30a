#!/bin/bash
# PC step with head-layer-1 init rows staged in LDS by the non-update waves: GPU suite, config-4 bench
# A/B against the previous commit (variants/old), SA-level phase trace (variants/satrace)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err &&
GENPOSE_HIP_LIB=variants/old/libgenpose_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_old.json 2> gpurun_out/bench_old.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_new2.json 2> gpurun_out/bench_new2.err &&
bash scripts/r2_satrace.sh
