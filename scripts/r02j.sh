#!/bin/bash
# r02j: observation kernel with chained blocks (o_nb*) and row-stream Windy knobs (w_*), A/B against the in-tree build.
set -o pipefail
mkdir -p gpurun_out
V=gym-cellular-automata_amd/gymca_amd/_lib/variants
for X in o_nb4 o_nb8; do
  GCA_LIB_PATH=$V/$X.so timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
    -p no:cacheprovider tests/test_gpu_observation.py > gpurun_out/r02j_pytest_$X.log 2>&1
  rc=$?; echo "pytest $X exit $rc"; tail -1 gpurun_out/r02j_pytest_$X.log; [ $rc -eq 0 ] || exit 1
done
bash scripts/ab.sh base o_nb2 o_nb4 o_nb8 && bash scripts/ab.sh o_nb8 o_nb4 o_nb2 base || exit 1
for W in base w_rd16 w_rd4 w_sh16 w_sh64 base; do
  if [ "$W" = base ]; then L=""; else L=$V/$W.so; fi
  GCA_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r02j_$W.json 2> gpurun_out/r02j_$W.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r02j_$W.json')); s=d['secondary']; c=d['config5']; print('$W', 'C2 ca_us', round(s['ca_kernel_ms']*1e3,2), 'of copy', round(s['ca_frac_of_same_size_copy'],3), '| C5 ca_us', round(c['ca_kernel_ms']*1e3,2), 'of copy', round(c['ca_frac_of_same_size_copy'],3))"
done
