#!/bin/bash
# Head-sequential layer 1 (layer 2 of the previous head in the MFMA gaps): GPU suite on the new build,
# config-4 bench A/B against the side-by-side build (variants/h1old), kernel trace of the new build
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/gputest.log 2>&1 &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err &&
GENPOSE_HIP_LIB=variants/h1old/libgenpose_hip.so timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_old.json 2> gpurun_out/bench_old.err &&
timeout -k 10 300 python bench.py --no-cpu-baseline > gpurun_out/bench_new2.json 2> gpurun_out/bench_new2.err &&
rm -rf gpurun_out/prof_c4 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o c4 -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --ode-calls 1 > gpurun_out/prof_c4.log 2>&1
