#!/bin/bash
# r02f: observation kernel rows-per-block / store-batching A/B
set -u
mkdir -p gpurun_out/r02f
timeout -k 10 300 python -u -m pytest tests/test_gpu_observation.py tests/test_gpu_batched_api.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r02f/pytest.log 2>&1 || exit 11
bash scripts/ab.sh base rb16 base rb16 > gpurun_out/r02f/ab.txt 2>&1 || exit 12
echo done > gpurun_out/r02f/done
