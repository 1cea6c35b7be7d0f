#!/bin/bash
# GPU session (r04): GPU tests on the in-tree library, the Windy tests on candidate variants, Windy env-step A/B,
# the headline profile (scripts/profile.sh) and the bench. Each step time-limited; a crash / abort / time limit ends
# the session. Usage (GPU box, repo root): bash scripts/gpu_session.sh <tag> "<windy variants>" [profile: 1|0]
TAG=$1; WV=$2; PROF=${3:-1}
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
RC=$?; echo "pytest exit $RC" >> $O/pytest_gpu.log
[ $RC -eq 0 ] || [ $RC -eq 1 ] || exit 20
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit 21
for v in $WV; do
  GCA_LIB_PATH=$V/$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_windy.py -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.log 2>&1
  RC=$?; echo "pytest exit $RC" >> $O/pytest_$v.log
  [ $RC -eq 0 ] || [ $RC -eq 1 ] || exit 22
done
for pass in 1 2 3; do
  [ -n "$WV" ] || break
  echo "windy $pass main $(timeout -k 10 120 python3 -u scripts/ab_windy_env.py)" >> $O/ab.txt || exit 23
  for v in $WV; do
    echo "windy $pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 120 python3 -u scripts/ab_windy_env.py)" >> $O/ab.txt || exit 24
  done
done
if [ "$PROF" = "1" ]; then bash scripts/profile.sh $TAG || exit 25; fi
timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 26
echo done > $O/done.txt
