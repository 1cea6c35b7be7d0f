#!/bin/bash
# SQ counters of the two Alexandridis step mappings (scripts/ab_march.py launches both), one rocprofv3 pass per counter
# set. Usage (repo root, GPU box): bash scripts/prof_ab_march.sh <tag>
set -u
TAG=${1:-march}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for PASS in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU" "FETCH_SIZE" "SQ_ACTIVE_INST_ANY SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE"; do
  N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $PASS -d $O/pmc_$N -o run --output-format csv -- python3 $R/scripts/ab_march.py > $O/pmc_$N.log 2>&1 || { echo "pmc pass $PASS failed: $?" >> $O/errors.txt; exit 12; }
done
echo done > $O/done.txt
