#!/bin/bash
# GPU session (r04): GPU tests on the in-tree library, candidate variants' kernel tests, the bench, and A/B timings of
# the marching step (scripts/ab_march.py) and the Windy env step (scripts/ab_windy_env.py) against variants.
# Usage (GPU box, repo root): bash scripts/gpu_ab3.sh <tag> "<march variants>" "<windy variants>"
TAG=$1; MV=$2; WV=$3
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
RC=$?; echo "pytest exit $RC" >> $O/pytest_gpu.log
[ $RC -eq 0 ] || [ $RC -eq 1 ] || exit 20
for v in $MV; do
  GCA_LIB_PATH=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_alex_march.py tests/test_gpu_alexandridis.py tests/test_gpu_observation.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1
  RC=$?; echo "pytest exit $RC" >> $O/pytest_$v.log
  [ $RC -eq 0 ] || [ $RC -eq 1 ] || exit 21
done
for v in $WV; do
  GCA_LIB_PATH=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_windy.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1
  RC=$?; echo "pytest exit $RC" >> $O/pytest_$v.log
  [ $RC -eq 0 ] || [ $RC -eq 1 ] || exit 21
done
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 22
for pass in 1 2 3; do
  echo "$pass main $(timeout -k 10 120 python3 -u scripts/ab_march.py --only march --reps 5)" >> $O/ab.txt || exit 23
  for v in $MV; do
    echo "$pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u scripts/ab_march.py --only march --reps 5)" >> $O/ab.txt || exit 24
  done
done
for pass in 1 2; do
  echo "512 $pass main $(timeout -k 10 180 python3 -u scripts/ab_march.py --size 512 --envs 1024 --reps 5)" >> $O/ab.txt || exit 25
  for v in $MV; do
    echo "512 $pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 180 python3 -u scripts/ab_march.py --size 512 --envs 1024 --reps 5)" >> $O/ab.txt || exit 26
  done
done
for pass in 1 2 3; do
  echo "windy $pass main $(timeout -k 10 120 python3 -u scripts/ab_windy_env.py)" >> $O/ab.txt || exit 27
  for v in $WV; do
    echo "windy $pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u scripts/ab_windy_env.py)" >> $O/ab.txt || exit 28
  done
done
echo done > $O/done.txt
