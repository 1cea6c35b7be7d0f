#!/bin/bash
# One rocprofv3 pass of VALU / wave / busy counters over scripts/ab_march.py (both Alexandridis mappings).
# Usage (repo root, GPU box): bash scripts/prof_valu.sh <tag>
set -u
TAG=${1:-valu}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- python3 $R/scripts/ab_march.py > $O/pmc.log 2>&1 || exit 12
python3 $R/scripts/pmc_kernels.py $O/pmc/run_counter_collection.csv
