#!/bin/bash
# One GPU session: GPU tests, smoke, bench, then (optionally) the profile. Each step time-limited;
# stops at the first failing step.
TAG=${1:-r01}
PROFILE=${2:-1}
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_gpu_$TAG.log 2>&1
echo "pytest exit $?" >> gpurun_out/pytest_gpu_$TAG.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$TAG.log 2>&1 || exit 21
timeout -k 10 500 python bench.py > gpurun_out/bench_$TAG.json 2> gpurun_out/bench_$TAG.err || exit 22
if [ "$PROFILE" = "1" ]; then bash scripts/profile.sh $TAG; fi
