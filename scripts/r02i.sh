#!/bin/bash
# r02i: row-stream Windy kernel (in-tree) vs the 16-cells-per-lane fast kernel (variant wold = -DGCA_WINDY_ROWS=0):
# the Windy GPU tests on the in-tree build, then the bench's Windy lines for both.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider \
  tests/test_gpu_windy.py tests/test_gpu_misc.py > gpurun_out/r02i_pytest.log 2>&1
rc=$?; echo "pytest exit $rc"; tail -3 gpurun_out/r02i_pytest.log; [ $rc -eq 0 ] || exit 1
for V in base wold base wold; do
  if [ "$V" = base ]; then L=""; else L=gym-cellular-automata_amd/gymca_amd/_lib/variants/$V.so; fi
  GCA_LIB_PATH=$L timeout -k 10 300 python bench.py --no-cpu-baseline --steps 20 > gpurun_out/r02i_$V.json 2> gpurun_out/r02i_$V.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/r02i_$V.json')); s=d['secondary']; c=d['config5']; print('$V', 'C2 ca_ms', round(s['ca_kernel_ms']*1e3,2), 'us frac', round(s['ca_roofline_frac'],3), 'of copy', round(s['ca_frac_of_same_size_copy'],3), 'env/s', round(s['env_steps_per_s']/1e6,2), 'M | C5 ca_ms', round(c['ca_kernel_ms']*1e3,2), 'us frac', round(c['ca_roofline_frac'],3), 'of copy', round(c['ca_frac_of_same_size_copy'],3), 'env/s', round(c['env_steps_per_s']/1e6,2), 'M')"
done
