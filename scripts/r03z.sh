#!/bin/bash
# r03z: in-place age stores skipped for lanes without FIRE / new fires (agest, the in-tree build) vs HEAD (base1):
# full GPU tests on the in-tree build, interleaved timing, FETCH / WRITE per variant (one counter per pass)
set -e
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=$R/gpurun_out/r03z
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_tree.log 2>&1
bash scripts/ab_rgb.sh $O 3 base1 agest
cd /tmp && export TMPDIR=/tmp
for v in base1 agest; do
  for c in FETCH_SIZE WRITE_SIZE; do
    GCA_LIB_PATH=$V/$v.so timeout -s KILL 120 rocprofv3 --pmc $c -d $O/pmc_${v}_$c -o run --output-format csv -- python3 $R/scripts/ab_march.py --only march --plain --reps 1 > $O/pmc_${v}_$c.log 2>&1
  done
done
echo done > $O/done.txt
