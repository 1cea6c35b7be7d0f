#!/bin/bash
# r02n: streaming observation kernel (GCA_OBS_STREAM = workgroup count) and 32-row Alexandridis tiles (th32 =
# -DGCA_ALEX_TH=32 -DGCA_ALEX_WGS=2) — GPU tests on the variants, then the headline A/B (obs = RGB observation kernel ms,
# fill = a write-only fill_ of the same buffer).
set -o pipefail
mkdir -p gpurun_out
V=gym-cellular-automata_amd/gymca_amd/_lib/variants
GCA_LIB_PATH=$V/os2048.so timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_observation.py tests/test_gpu_batched_api.py > gpurun_out/r02n_pytest.log 2>&1
rc=$?; echo "pytest os2048 exit $rc"; tail -n 1 gpurun_out/r02n_pytest.log; [ $rc -eq 0 ] || exit 1
GCA_LIB_PATH=$V/th32.so timeout -k 10 400 python -u -m pytest -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_alexandridis.py tests/test_gpu_edge_slope.py -k "not tile_skip" > gpurun_out/r02n_pytest_th32.log 2>&1
rc=$?; echo "pytest th32 exit $rc"; tail -n 3 gpurun_out/r02n_pytest_th32.log; [ $rc -le 1 ] || exit 1
bash scripts/ab.sh base os1024 os2048 os4096 os8192 th32 && bash scripts/ab.sh th32 os8192 os2048 base
