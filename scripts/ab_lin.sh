#!/bin/bash
# Same-box A/B of library variants on the split token linears (scripts/lin_bench.py) and, with PW=1, on the
# DINO-pointwise config-4 step (bench.py --dino pointwise): alternating rounds, bit-identity via the digests.
# usage: scripts/ab_lin.sh ROUNDS LIB1 LIB2 ...
ROUNDS=$1; shift
for r in $(seq 1 "$ROUNDS"); do
  for L in "$@"; do
    echo "# round $r $L"
    GENPOSE_HIP_LIB=$L timeout -k 10 300 python scripts/lin_bench.py || exit 1
    if [ "${PW:-0}" = 1 ]; then
      GENPOSE_HIP_LIB=$L timeout -k 10 300 python bench.py --dino pointwise --steps 5 --warmup 2 --no-cpu-baseline \
        --ode-calls 0 --f32-steps 0 --pointwise-steps 0 > gpurun_out/ab_lin_pw.json || exit 1
      python -c "import json;d=json.load(open('gpurun_out/ab_lin_pw.json'));print('pointwise', round(d['ms_per_step'],3), 'sampler', round(d['roofline']['sampler_ms_per_step'],3))"
    fi
  done
done
