#!/bin/bash
# Head-layer-1 init loads: update waves after the update; other waves at entry (default) or right before
# the trunk (variants/late, PC_HINIT_LATE); A/B against the previous commit (variants/old), phase traces
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err &&
GENPOSE_HIP_LIB=variants/late/libgenpose_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_late.json 2> gpurun_out/bench_late.err &&
GENPOSE_HIP_LIB=variants/old/libgenpose_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_old.json 2> gpurun_out/bench_old.err &&
GENPOSE_HIP_LIB=variants/trace_new/libgenpose_hip.so timeout -k 10 120 python scripts/pc_trace.py 256 50 > gpurun_out/trace_new.json 2>&1 &&
GENPOSE_HIP_LIB=variants/trace_late/libgenpose_hip.so timeout -k 10 120 python scripts/pc_trace.py 256 50 > gpurun_out/trace_late.json 2>&1
