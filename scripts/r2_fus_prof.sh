#!/bin/bash
# Fused-encoder timing (B=256) and its kernel breakdown
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python scripts/enc_bench.py 256 5 > gpurun_out/enc_bench.json 2> gpurun_out/enc_bench.err &&
rm -rf gpurun_out/prof_fus &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fus -o fus -- python3 scripts/enc_bench.py 256 2 > gpurun_out/prof_fus.log 2>&1
