#!/bin/bash
# PC-step phase trace at config 4 (64-candidate tiles) with the trace build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
export GENPOSE_HIP_LIB=variants/trace/libgenpose_hip.so
timeout -k 10 120 python scripts/pc_trace.py 256 50 > gpurun_out/trace_nt4.json 2>&1
