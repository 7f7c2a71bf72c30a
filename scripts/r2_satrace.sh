#!/bin/bash
# Phase trace of the split-f16 SA levels 2-3 at B=256 (trace build), after the level-3 6-tile blocks
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
GENPOSE_HIP_LIB=variants/satrace/libgenpose_hip.so timeout -k 10 120 python scripts/split_trace.py 256 > gpurun_out/split_trace_b256.json 2>&1
