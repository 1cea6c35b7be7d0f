#!/bin/bash
# A/B the headline kernel across slope layouts in one GPU session: bash scripts/ab_layout.sh packed edge ...
mkdir -p gpurun_out
for L in "$@"; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --headline-only --steps 40 --slope-layout $L > gpurun_out/abl_$L.json 2> gpurun_out/abl_$L.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abl_$L.json')); r=d['roofline']; print('$L', round(r['kernel_ms'],4), 'ms', round(d['value']/1e9,2), 'Gcell/s', round(r['moved_gbs']), 'GB/s moved')"
done
