#!/bin/bash
# r02o: direct observation kernel (GCA_OBS_DIRECT: no LDS transposition, 768-B dwordx3 stores, nt / plain) — observation
# GPU tests on the variant, then the headline A/B (obs = RGB observation kernel ms, fill = write-only fill_ of the buffer).
set -o pipefail
mkdir -p gpurun_out
V=gym-cellular-automata_amd/gymca_amd/_lib/variants
GCA_LIB_PATH=$V/od1.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_observation.py tests/test_gpu_batched_api.py > gpurun_out/r02o_pytest.log 2>&1
rc=$?; echo "pytest od1 exit $rc"; tail -n 1 gpurun_out/r02o_pytest.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab.sh base od1 od1nt0 os2048 && bash scripts/ab.sh os2048 od1nt0 od1 base
