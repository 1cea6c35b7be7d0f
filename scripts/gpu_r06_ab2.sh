#!/bin/bash
# r06: full GPU suite on the in-tree library, then main vs <variant> on the mid-episode and the reset (episode-start)
# states, plain and fused frame, two interleaved passes. Usage: bash scripts/gpu_r06_ab2.sh <tag> <variant>
TAG=$1; V=$2
O=gpurun_out/$TAG
L=gym-cellular-automata_amd/gymca_amd/_lib/variants/$V.so
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_all.log 2>&1 || exit 10
for pass in 1 2; do
  for st in "" "--reset"; do
    echo "pass $pass main $st $(timeout -k 10 180 python3 -u scripts/ab_march.py --only march --reps 5 $st)" >> $O/ab.txt || exit 21
    echo "pass $pass $V $st $(GCA_LIB_PATH=$L timeout -k 10 180 python3 -u scripts/ab_march.py --only march --reps 5 $st)" >> $O/ab.txt || exit 22
  done
done
echo done > $O/done.txt
