#!/bin/bash
# r02h: LDS-DMA slope loads in the packed Alexandridis step (variant gl1 = -DGCA_ALEX_GLDS=1).
# Parity of the variant on the packed-kernel tests, then the headline A/B against the in-tree build.
set -o pipefail
mkdir -p gpurun_out
V=gym-cellular-automata_amd/gymca_amd/_lib/variants
for X in "$@"; do
  GCA_LIB_PATH=$V/$X.so timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
    -p no:cacheprovider tests/test_gpu_edge_slope.py -k "packed or tile_skip" > gpurun_out/r02h_pytest_$X.log 2>&1
  rc=$?; echo "pytest $X exit $rc"; tail -3 gpurun_out/r02h_pytest_$X.log
  [ $rc -eq 0 ] || exit 1
done
bash scripts/ab.sh base "$@" && bash scripts/ab.sh "$@" base
