#!/bin/bash
# Split trunk with act2 separate from act1 (layer-2 partials aliased onto act1: one barrier fewer),
# LDS-only barriers, init loads in the pose_encoder.0 phase: GPU suite, config-4 bench A/B against the
# previous commit (variants/old), PC-step phase trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err &&
GENPOSE_HIP_LIB=variants/old/libgenpose_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_old.json 2> gpurun_out/bench_old.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_new2.json 2> gpurun_out/bench_new2.err &&
GENPOSE_HIP_LIB=variants/trace_new/libgenpose_hip.so timeout -k 10 120 python scripts/pc_trace.py 256 50 > gpurun_out/trace_new.json 2>&1
