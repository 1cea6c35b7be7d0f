#!/bin/bash
# r02r: wave-priority hook on the Alexandridis step (pr1 = -DGCA_ALEX_PRIO=1: priority 3 while a tile issues its
# staging loads; pr2 = 2: also for the stores; pr3 = 3: also 2 for the direction pass); pr4 / pr5 = 4 / 5) — packed-kernel GPU tests on pr4,
# then the headline A/B.
set -o pipefail
mkdir -p gpurun_out
V=gym-cellular-automata_amd/gymca_amd/_lib/variants
GCA_LIB_PATH=$V/pr4.so timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
  -p no:cacheprovider tests/test_gpu_edge_slope.py tests/test_gpu_alexandridis.py -k "packed or tile_skip or chi_square" > gpurun_out/r02r_pytest.log 2>&1
rc=$?; echo "pytest pr4 exit $rc"; tail -n 1 gpurun_out/r02r_pytest.log; [ $rc -eq 0 ] || exit 1
bash scripts/ab.sh base pr1 pr4 pr5 && bash scripts/ab.sh pr5 pr4 pr1 base && bash scripts/ab.sh base pr1 pr4 pr5
python -c "import json; print('traffic', json.load(open('gpurun_out/ab_base.json'))['roofline']['traffic'])"
