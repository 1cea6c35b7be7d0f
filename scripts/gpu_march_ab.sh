#!/bin/bash
# Marching-kernel A/B of candidate library builds against the in-tree one (GPU box, repo root): the march /
# Alexandridis / observation GPU tests on each candidate, three interleaved passes of scripts/ab_march.py (plain and
# fused-frame step, 4096 x 256^2), two of the reset state and of 1024 x 512^2, then per build one rocprofv3 pass each of FETCH_SIZE, WRITE_SIZE and the VALU
# counters over the plain step. Each step time-limited; a failure ends the run.
# Usage: [SKIP_TESTS=1] bash scripts/gpu_march_ab.sh <tag> "<variants>"
TAG=$1; MV=$2
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=$R/gpurun_out/$TAG
mkdir -p $O
for v in $MV; do
  [ -n "$SKIP_TESTS" ] && break  # timing-only probes (e.g. a tile height the activity-map tests do not fit)
  GCA_LIB_PATH=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_alex_march.py tests/test_gpu_alexandridis.py tests/test_gpu_observation.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1
  RC=$?; echo "pytest exit $RC" >> $O/pytest_$v.log
  [ $RC -eq 0 ] || exit 21
done
for pass in 1 2 3; do
  echo "$pass main $(timeout -k 10 120 python3 -u scripts/ab_march.py --only march --reps 5)" >> $O/ab.txt || exit 23
  for v in $MV; do
    echo "$pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u scripts/ab_march.py --only march --reps 5)" >> $O/ab.txt || exit 24
  done
done
for pass in 1 2; do
  echo "reset $pass main $(timeout -k 10 120 python3 -u scripts/ab_march.py --only march --plain --reset --reps 5)" >> $O/ab.txt || exit 25
  for v in $MV; do
    echo "reset $pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u scripts/ab_march.py --only march --plain --reset --reps 5)" >> $O/ab.txt || exit 26
  done
  echo "512 $pass main $(timeout -k 10 180 python3 -u scripts/ab_march.py --only march --size 512 --envs 1024 --reps 5)" >> $O/ab.txt || exit 27
  for v in $MV; do
    echo "512 $pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 180 python3 -u scripts/ab_march.py --only march --size 512 --envs 1024 --reps 5)" >> $O/ab.txt || exit 28
  done
done
cd /tmp && export TMPDIR=/tmp
for v in main $MV; do
  L=$R/gym-cellular-automata_amd/gymca_amd/_lib/libgca_hip.so
  [ $v = main ] || L=$V/$v.so
  for PASS in "FETCH_SIZE" "WRITE_SIZE" "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES GRBM_GUI_ACTIVE"; do
    N=$(echo $PASS | cut -d' ' -f1)
    GCA_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $PASS -d $O/pmc_$v/$N -o run --output-format csv -- python3 $R/scripts/ab_march.py --only march --plain --reps 2 > $O/pmc_${v}_$N.log 2>&1 || exit 30
  done
done
echo done > $O/done.txt
