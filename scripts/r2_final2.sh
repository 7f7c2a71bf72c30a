#!/bin/bash
# Round-2 closing measurement (scripts/r2_final.sh) + level-3 tile-width probe (variants/ct3_{3,2}:
# 48 / 32 columns per workgroup, two / three workgroups per CU) + SA-level phase trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
bash scripts/r2_final.sh &&
timeout -k 10 200 python scripts/enc_bench.py 256 10 > gpurun_out/enc_ct6.json 2> gpurun_out/enc_ct6.err &&
GENPOSE_HIP_LIB=variants/ct3_3/libgenpose_hip.so timeout -k 10 200 python scripts/enc_bench.py 256 10 > gpurun_out/enc_ct3.json 2> gpurun_out/enc_ct3.err &&
GENPOSE_HIP_LIB=variants/ct3_2/libgenpose_hip.so timeout -k 10 200 python scripts/enc_bench.py 256 10 > gpurun_out/enc_ct2.json 2> gpurun_out/enc_ct2.err &&
bash scripts/r2_satrace.sh
