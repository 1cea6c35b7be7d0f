#!/bin/bash
# GPU session (r05): A/B of the marching step against variants built by scripts/build_variant.sh -- the march tests
# on each variant, interleaved timing passes (scripts/ab_march.py), and one FETCH_SIZE / WRITE_SIZE pass per build.
# Each step time-limited; a crash / abort / time limit ends the session.
# Usage (GPU box, repo root): bash scripts/gpu_variant_ab.sh <tag> "<variants>"
TAG=$1; VARS=$2
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in $VARS; do
  GCA_LIB_PATH=$V/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_alex_march.py tests/test_gpu_alex_draws.py tests/test_gpu_observation.py -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1
  RC=$?; echo "pytest exit $RC" >> $O/pytest_$v.log
  [ $RC -eq 0 ] || [ $RC -eq 1 ] || exit 20
done
for pass in 1 2 3; do
  echo "pass $pass main $(timeout -k 10 180 python3 -u scripts/ab_march.py --only march --reps 5)" >> $O/ab.txt || exit 21
  for v in $VARS; do
    echo "pass $pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 180 python3 -u scripts/ab_march.py --only march --reps 5)" >> $O/ab.txt || exit 22
  done
done
cd /tmp && export TMPDIR=/tmp
for v in main $VARS; do
  LP=""; [ "$v" = "main" ] || LP=$V/$v.so
  for PASS in FETCH_SIZE WRITE_SIZE; do
    GCA_LIB_PATH=$LP timeout -k 10 300 rocprofv3 --pmc $PASS -d $O/pmc_${v}_$PASS -o run --output-format csv -- python3 $R/scripts/ab_march.py --only march --plain --reps 2 > $O/pmc_${v}_$PASS.log 2>&1 || echo "pmc $v $PASS failed: $?" >> $O/errors.txt
  done
done
echo done > $O/done.txt
