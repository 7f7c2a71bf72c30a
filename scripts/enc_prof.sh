#!/bin/bash
# Kernel trace of the encoder timing sweep (scripts/kbench.py --enc) -> gpurun_out/prof_enc
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
rm -rf gpurun_out/prof_enc
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_enc -o enc -- python3 scripts/kbench.py --enc > gpurun_out/kb_enc.json 2>&1
