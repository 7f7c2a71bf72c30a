#!/bin/bash
# Encoder A/B: narrow-level gather pipeline + wide split column blocks (main) against HEAD's build and
# two variants (enc_a: 64-column split blocks; enc_b: level-3 ring depth 1); encoder GPU tests first.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "encoder or sa_level or large_rows or fusion" > gpurun_out/gputest_enc.log 2>&1 &&
for v in head enc_a enc_b; do
  GENPOSE_HIP_LIB=variants/$v/libgenpose_hip.so timeout -k 10 200 python scripts/enc_bench.py 256 10 > gpurun_out/enc_$v.json 2> gpurun_out/enc_$v.err || exit 1
done &&
timeout -k 10 200 python scripts/enc_bench.py 256 10 > gpurun_out/enc_main.json 2> gpurun_out/enc_main.err &&
rm -rf gpurun_out/prof_enc &&
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_enc -o enc -- python3 scripts/enc_bench.py 256 3 > gpurun_out/prof_enc.log 2>&1
