#!/bin/bash
# PC-step phase trace (trace build) + default bench line (no CPU baseline)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GENPOSE_HIP_LIB=variants/trace/libgenpose_hip.so timeout -k 10 120 python scripts/pc_trace.py 256 50 > gpurun_out/trace_nt4.json 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_nocpu.json 2> gpurun_out/bench_nocpu.err
