#!/bin/bash
# Profile the bench workload on the GPU box: kernel trace + stats, then HBM and SQ counters,
# each in its own rocprofv3 run (never --pmc together with runtime/sys traces).
# Usage (from the repo root on the GPU box): bash scripts/profile.sh <tag>
set -u
TAG=${1:-r01}
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/prof_$TAG
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
B="python3 $R/bench.py --no-cpu-baseline --headline-only"
timeout -k 10 120 rocprofv3 -L > $O/counters_available.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/trace -o run --output-format csv -- $B --steps 20 --warmup 20 --no-secondary > $O/trace.log 2>&1 || exit 11
for PASS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU"; do
  N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -k 10 400 rocprofv3 --pmc $PASS -d $O/pmc_$N -o run --output-format csv -- $B --steps 4 --warmup 1 --no-secondary > $O/pmc_$N.log 2>&1 || echo "pmc pass $PASS failed: $?" >> $O/errors.txt
done
echo profile done > $O/done.txt
