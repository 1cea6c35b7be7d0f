#!/bin/bash
# r02k: plain observation kernel (no staging) — observation + env GPU tests on the in-tree build, then the headline
# A/B (obs = RGB observation kernel ms) against the staged kernel (op0) and chunk-per-wave knobs.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_observation.py tests/test_gpu_batched_api.py > gpurun_out/r02k_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -1 gpurun_out/r02k_pytest.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab.sh base op0 op4 op16 && bash scripts/ab.sh op16 op4 op0 base
