#!/bin/bash
# Encoder parity tests + encoder-only timing + kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "encoder or sa_level or fus or large or golden" > gpurun_out/gputest_enc.log 2>&1 &&
timeout -k 10 200 python scripts/enc_bench.py 256 5 > gpurun_out/enc_bench.json 2> gpurun_out/enc_bench.err &&
rm -rf gpurun_out/prof_enc &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enc -o enc -- python3 scripts/enc_bench.py 256 2 > gpurun_out/prof_enc.log 2>&1
