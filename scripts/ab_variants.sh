#!/bin/bash
# A/B of marching-kernel build variants (scripts/build_variant.sh) on the GPU box: interleaved timing passes of
# scripts/ab_march.py (march only, plain step) and one PMC pass per variant (VALU instructions, busy cycles).
# Usage: bash scripts/ab_variants.sh <out_dir> <variant names...>; results in <out_dir>/ab.txt and <out_dir>/pmc_<v>/.
set -e
OUT=$(realpath -m $1); shift
R=$(cd "$(dirname "$0")/.." && pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
mkdir -p $OUT
for pass in 1 2; do
  for v in "$@"; do
    echo "$pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u $R/scripts/ab_march.py --only march --plain --reps 5)" | tee -a $OUT/ab.txt
  done
done
cd /tmp && export TMPDIR=/tmp
for v in "$@"; do
  GCA_LIB_PATH=$V/$v.so timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES -d $OUT/pmc_$v -o run --output-format csv -- python3 $R/scripts/ab_march.py --only march --plain --reps 1 > $OUT/pmc_$v.log 2>&1
  echo "pmc $v done"
done
