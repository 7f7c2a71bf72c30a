#!/bin/bash
# A/B: encoder of batch k+1 overlapped with the sampler of batch k (bench.py --pipeline 1) vs serial
set -o pipefail
cd $GRAFT_REPO_ROOT
for c in 2 4; do
  for p in 0 1; do
    timeout -k 10 200 python bench.py --config $c --steps 5 --warmup 2 --no-cpu-baseline --pipeline $p > gpurun_out/pipe_c${c}_p${p}.log 2>&1 || exit 1
  done
done
timeout -k 10 200 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pred_func or smoke or pipeline" > gpurun_out/t_pipe.log 2>&1
