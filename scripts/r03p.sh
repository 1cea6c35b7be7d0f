#!/bin/bash
# r03p: fire-ring order / packed constants (new1) and the tile-major wave order (chNNN) vs the HEAD build (base0)
set -e
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=$R/gpurun_out/r03p
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_alex_march.py tests/test_gpu_observation.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_new1.log 2>&1
GCA_LIB_PATH=$V/ch256.so timeout -k 10 300 python -u -m pytest tests/test_gpu_alex_march.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_ch256.log 2>&1
bash scripts/ab_rgb.sh $O 2 base0 new1 ch128 ch256 ch512
cd /tmp && export TMPDIR=/tmp
for v in base0 new1 ch256 ch512; do
  GCA_LIB_PATH=$V/$v.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE WRITE_SIZE -d $O/pmc_$v -o run --output-format csv -- python3 $R/scripts/ab_march.py --only march --plain --reps 1 > $O/pmc_$v.log 2>&1
done
echo done > $O/done.txt
