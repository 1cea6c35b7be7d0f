#!/bin/bash
# A/B of marching-kernel build variants, plain and fused-frame step (scripts/ab_march.py --only march), interleaved
# passes. Usage (GPU box): bash scripts/ab_rgb.sh <out_dir> <passes> <variant names...>; results in <out_dir>/ab.txt
set -e
OUT=$(realpath -m $1); shift
P=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
mkdir -p $OUT
for pass in $(seq $P); do
  for v in "$@"; do
    echo "$pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u $R/scripts/ab_march.py --only march --reps 5)" | tee -a $OUT/ab.txt
  done
done
