#!/bin/bash
# Split-encoder trace: gather prefetch (D=2) and D=3 ring, plus encoder tests on the default build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "encoder or sa_level or large_rows" > gpurun_out/gputest_enc.log 2>&1 &&
GENPOSE_HIP_LIB=variants/satrace/libgenpose_hip.so timeout -k 10 180 python scripts/split_trace.py 256 > gpurun_out/split_trace_d2.json 2>&1 &&
GENPOSE_HIP_LIB=variants/satrace_d3/libgenpose_hip.so timeout -k 10 180 python scripts/split_trace.py 256 > gpurun_out/split_trace_d3.json 2>&1 &&
timeout -k 10 200 python scripts/enc_bench.py 256 5 > gpurun_out/enc_bench.json 2> gpurun_out/enc_bench.err
