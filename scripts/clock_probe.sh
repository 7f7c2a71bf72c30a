#!/bin/bash
# Poll the shader clock while scripts/clock_probe.py MODE runs (calibration aid): amd-smi / rocm-smi readings
# once a second, then the workload's own per-window rates.   usage: scripts/clock_probe.sh MODE [SECONDS]
MODE=$1; SECS=${2:-8}
timeout -k 10 120 python scripts/clock_probe.py "$MODE" "$SECS" > gpurun_out/clock_${MODE}.json 2>&1 &
P=$!
sleep 12
for i in $(seq 1 6); do
  echo "t+$i: $(timeout 10 rocm-smi --showclocks 2>/dev/null | grep -E 'sclk|fclk|mclk' | tr -s ' ' | tr '\n' ';')"
  sleep 1
done
wait $P; rc=$?
cat gpurun_out/clock_${MODE}.json
exit $rc
