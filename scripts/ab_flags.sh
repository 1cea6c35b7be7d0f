#!/bin/bash
# A/B bench.py flag sets in one GPU session: bash scripts/ab_flags.sh "" "--tile-skip" ...
mkdir -p gpurun_out
i=0
for F in "$@"; do
  i=$((i+1))
  timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --steps 40 $F > gpurun_out/abf_$i.json 2> gpurun_out/abf_$i.err || exit 1
  python -c "import json; d=json.load(open('gpurun_out/abf_$i.json')); r=d['roofline']; print('[$F]', round(r['kernel_ms'],4), 'ms', 'episode', round(d['episode_start']['kernel_ms'],4))"
done
