#!/bin/bash
# PC tests + PC trace + bench + split-encoder trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/r2_pc_iter.sh &&
GENPOSE_HIP_LIB=variants/satrace/libgenpose_hip.so timeout -k 10 180 python scripts/split_trace.py 256 > gpurun_out/split_trace.json 2>&1
