#!/bin/bash
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export GENPOSE_HIP_LIB=variants/trace/libgenpose_hip.so
timeout -k 10 120 python scripts/pc_trace.py 256 50 > gpurun_out/trace_nt4.json 2>&1 &&
timeout -k 10 120 python scripts/pc_trace.py 64 50 > gpurun_out/trace_nt1.json 2>&1 &&
timeout -k 10 120 python scripts/pc_trace.py 96 50 > gpurun_out/trace_nt2.json 2>&1
