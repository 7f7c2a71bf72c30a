#!/bin/bash
# Multi-process determinism matrix for the encoder (scripts/race_probe.py levels modes): each arm runs
# PROCS processes that each encode their batch REPS times on recycled memory and compare every level with
# their first repetition; one summary line per arm in gpurun_out/race_matrix.txt.
# usage: bash scripts/race_matrix.sh PROCS REPS ARM [ARM ...]
#   ARM = name:mode[:lib-variant][:env NAME=VALUE]   e.g. base:levels  sync:levels:sync  geom:levels_geom
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
PROCS=$1; REPS=$2; shift 2
mkdir -p gpurun_out
for arm in "$@"; do
  IFS=':' read -r name mode lib envkv <<< "$arm"
  out=gpurun_out/race_$name
  mkdir -p $out
  (
    [ -n "$lib" ] && export GENPOSE_HIP_LIB=$GRAFT_REPO_ROOT/variants/$lib/libgenpose_hip.so
    [ -n "$envkv" ] && export "$envkv"
    timeout -k 10 240 python -u scripts/race_probe.py --mode "$mode" --procs "$PROCS" --reps "$REPS" --outdir $out \
      > $out/log.txt 2>&1
  )
  rc=$?
  echo "$name rc=$rc $(tail -n 1 $out/log.txt)" | tee -a gpurun_out/race_matrix.txt
  [ $rc -ne 0 ] && exit $rc
done
exit 0
