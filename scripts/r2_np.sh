#!/bin/bash
# Level-0 narrow launch probes: FPS side only / branch a only / branch b only (timing only)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
for v in 1 2 3; do
  rm -rf gpurun_out/prof_np$v
  GENPOSE_HIP_LIB=variants/np$v/libgenpose_hip.so timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_np$v -o np -- python3 scripts/enc_bench.py 256 3 > gpurun_out/np$v.log 2>&1 || exit 1
done
