#!/bin/bash
# r06 GPU session: the new parity tests, then an A/B of variant builds against the in-tree library
# (scripts/gpu_variant_ab.sh). Each step time-limited; a crash / abort / time limit ends the session.
# Usage (GPU box, repo root): bash scripts/gpu_r06.sh <tag> "<variants>" "<test files>"
TAG=$1; VARS=$2; TESTS=$3
O=gpurun_out/$TAG
mkdir -p $O
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread $TESTS > $O/pytest.log 2>&1 || exit 10
fi
if [ -n "$VARS" ]; then
  bash scripts/gpu_variant_ab.sh $TAG "$VARS" || exit $?
fi
echo session done > $O/session_done.txt
