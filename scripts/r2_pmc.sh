#!/bin/bash
# PMC passes of the config-4 PC step (12,800 rows: 64-candidate split tiles)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
rm -rf gpurun_out/pmc_c4
bash scripts/pmc_passes.sh gpurun_out/pmc_c4 256 > gpurun_out/pmc_c4.log 2>&1 &&
python scripts/pmc_pc_json.py gpurun_out/pmc_c4 12800 > gpurun_out/pmc_pc_step_config4.json
