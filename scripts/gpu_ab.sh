#!/bin/bash
# One GPU session: GPU tests, smoke, bench, then A/B timings of the marching step against library variants
# (scripts/build_variant.sh) and the W = 512 march vs tiled comparison. Each step time-limited; stops at the first
# failing step. Usage (GPU box, repo root): bash scripts/gpu_ab.sh <tag> [variant names...]
TAG=${1:-r04}; shift
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
RC=$?
echo "pytest exit $RC" >> $O/pytest_gpu.log
# 1 = some test failed (read the log, go on measuring); anything else (crash, abort, time limit): stop here
[ $RC -eq 0 ] || [ $RC -eq 1 ] || exit 20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 21
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 22
for pass in 1 2; do
  echo "$pass new $(timeout -k 10 120 python3 -u scripts/ab_march.py --only march --plain --reps 5)" >> $O/ab.txt || exit 23
  for v in "$@"; do
    echo "$pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u scripts/ab_march.py --only march --plain --reps 5)" >> $O/ab.txt || exit 24
  done
done
echo "512 new $(timeout -k 10 180 python3 -u scripts/ab_march.py --size 512 --envs 1024 --reps 5)" >> $O/ab.txt || exit 25
echo done > $O/done.txt
