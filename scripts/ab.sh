#!/bin/bash
# A/B the headline kernel across library variants: bash scripts/ab.sh <variant-name>...
# ("base" = the in-tree libgca_hip.so). One bench line per variant into gpurun_out/ab_<name>.json.
# AB_ARGS: extra bench flags (e.g. "--headline-only" for the headline kernel alone).
mkdir -p gpurun_out
for V in "$@"; do
  if [ "$V" = base ]; then L=""; else L=gym-cellular-automata_amd/gymca_amd/_lib/variants/$V.so; fi
  GCA_LIB_PATH=$L timeout -k 10 240 python bench.py --no-cpu-baseline --no-secondary --steps 30 $AB_ARGS > gpurun_out/ab_$V.json 2> gpurun_out/ab_$V.err || exit 1
  python -c "
import json
d = json.load(open('gpurun_out/ab_$V.json')); r = d['roofline']
rgb = d.get('with_rgb_observation') or {}
ep = d.get('episode_start') or {}
print('$V', round(r['kernel_ms'], 4), 'ms', round(d['value'] / 1e9, 2), 'Gcell/s', 'episode', ep.get('kernel_ms'),
      'rgb_step_ms', rgb.get('ms_per_step'), 'rgb_kernels_ms', rgb.get('step_and_frame_kernels_ms'))"
done
