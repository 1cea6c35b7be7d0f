#!/bin/bash
# r02e: observation kernel head rework — GPU parity tests, then A/B against HEAD's build.
set -u
mkdir -p gpurun_out/r02e
timeout -k 10 300 python -u -m pytest tests/test_gpu_observation.py tests/test_gpu_batched_api.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02e/pytest.log 2>&1 || exit 11
bash scripts/ab.sh base head rb16 base head rb16 > gpurun_out/r02e/ab.txt 2>&1 || exit 12
echo done > gpurun_out/r02e/done
