#!/bin/bash
# A/B the headline kernel across library variants: bash scripts/ab.sh <variant-name>...
# ("base" = the in-tree libgca_hip.so). One bench line per variant into gpurun_out/ab_<name>.json.
mkdir -p gpurun_out
for V in "$@"; do
  if [ "$V" = base ]; then L=""; else L=gym-cellular-automata_amd/gymca_amd/_lib/variants/$V.so; fi
  GCA_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --steps 30 > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || exit 1
  python -c "import json,sys; d=json.load(open('gpurun_out/ab_$V.json')); r=d['roofline']; print('$V', round(r['kernel_ms'],4), 'ms', round(d['value']/1e9,2), 'Gcell/s', round(r['frac'],4), 'episode', round(d['episode_start']['kernel_ms'],4), 'obs', round(d['with_rgb_observation']['obs_kernel_ms'],4), 'fill', round(d['with_rgb_observation'].get('same_buffer_fill_ms',0),4))"
done
