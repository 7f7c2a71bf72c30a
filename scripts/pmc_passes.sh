#!/bin/bash
# PMC passes (one counter group per run, --pmc only, as MI355X_MICROARCH.md prescribes).
# usage: bash scripts/pmc_passes.sh OUTDIR [rows-arg]
set -u
OUT=$1; shift
export TMPDIR=/tmp
mkdir -p $OUT
i=0
for grp in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F32 GRBM_GUI_ACTIVE" \
           "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU"; do
  i=$((i+1))
  timeout -k 10 240 rocprofv3 --pmc $grp -d $OUT/p$i -o pass$i --output-format csv -- python scripts/pmc_target.py "$@" > $OUT/p$i.log 2>&1 || { echo "pass $i failed rc=$?"; exit 1; }
done
echo done
