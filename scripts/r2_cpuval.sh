#!/bin/bash
# Full GPU suite + the CPU-baseline sample checked against the full 256-object batch on the GPU host
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 900 python -u scripts/cpu_full_vs_sample.py > gpurun_out/cpu_full_vs_sample.json 2> gpurun_out/cpu_full_vs_sample.err
