#!/bin/bash
# Windy CA-only A/B (scripts/ab_windy_ca.py) of candidate builds against the in-tree one, after the Windy GPU tests on
# each candidate. Each step time-limited; a failure ends the run. Usage (GPU box): bash scripts/gpu_windy_ca_ab.sh <tag> "<variants>"
TAG=$1; WV=$2
V=$(pwd)/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=gpurun_out/$TAG
mkdir -p $O
for v in $WV; do
  GCA_LIB_PATH=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_windy.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1
  RC=$?; echo "pytest exit $RC" >> $O/pytest_$v.log
  [ $RC -eq 0 ] || exit 22
done
for pass in 1 2 3; do
  echo "ca $pass main $(timeout -k 10 120 python3 -u scripts/ab_windy_ca.py)" >> $O/ab.txt || exit 23
  for v in $WV; do
    echo "ca $pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u scripts/ab_windy_ca.py)" >> $O/ab.txt || exit 24
  done
done
echo done > $O/done.txt
