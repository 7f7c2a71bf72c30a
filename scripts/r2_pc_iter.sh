#!/bin/bash
# PC-step iteration: PC/ODE golden + large-row tests, phase trace, bench line
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "pc_ or ode or golden or philox or abi or tracking" > gpurun_out/gputest_pc.log 2>&1 &&
GENPOSE_HIP_LIB=variants/trace/libgenpose_hip.so timeout -k 10 120 python scripts/pc_trace.py 256 50 > gpurun_out/trace_nt4.json 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_nocpu.json 2> gpurun_out/bench_nocpu.err
