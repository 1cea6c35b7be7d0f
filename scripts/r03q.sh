#!/bin/bash
# r03q: grid-code ring + plane-3 skip (new2, the in-tree build) vs the HEAD build (base0) and new1 (ring order only):
# march / observation tests, interleaved timing, FETCH_SIZE per variant (one counter per pass)
set -e
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=$R/gpurun_out/${TAG:-r03q}
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_alex_march.py tests/test_gpu_observation.py tests/test_gpu_alexandridis.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_tree.log 2>&1
bash scripts/ab_rgb.sh $O 3 base0 new1 new4
cd /tmp && export TMPDIR=/tmp
for v in new4; do
  for c in FETCH_SIZE WRITE_SIZE; do
    GCA_LIB_PATH=$V/$v.so timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc_${v}_$c -o run --output-format csv -- python3 $R/scripts/ab_march.py --only march --plain --reps 1 > $O/pmc_${v}_$c.log 2>&1
  done
done
echo done > $O/done.txt
