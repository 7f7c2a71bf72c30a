set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_nt2final.log 2>&1 &&
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/smoke_nt2.log 2>&1 &&
timeout -k 10 240 python bench.py --config 4 --steps 5 --warmup 2 > gpurun_out/bench_config4_nt2.log 2>&1 &&
timeout -k 10 240 python bench.py --config 5 --steps 3 --warmup 1 > gpurun_out/bench_config5_nt2.log 2>&1 &&
timeout -k 10 240 python bench.py --config 3 --steps 5 --warmup 2 > gpurun_out/bench_config3_nt2.log 2>&1 &&
cd /tmp && export TMPDIR=/tmp && timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_c4 -o c4 -- python3 $GRAFT_REPO_ROOT/bench.py --config 4 --steps 3 --warmup 1 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof_c4.log 2>&1
