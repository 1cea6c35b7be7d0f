#!/bin/bash
# A/B the Windy CA kernel (BASELINE config 2 CA-only, 1024 x 256^2) across library variants:
# bash scripts/ab_windy.sh <variant-name>...  ("base" = the in-tree libgca_hip.so)
mkdir -p gpurun_out
for V in "$@"; do
  if [ "$V" = base ]; then L=""; else L=gym-cellular-automata_amd/gymca_amd/_lib/variants/$V.so; fi
  GCA_LIB_PATH=$L timeout -k 10 240 python -c "
import argparse, json, sys, torch
sys.argv = ['bench.py']
import bench
args = bench.parse(); args.steps = 200
world, rank, device, pg = bench.setup_dist(args)
r = bench.bench_windy(args, world, rank, device, pg)
print('$V', round(r['ca_kernel_ms'] * 1e3, 2), 'us', round(r['ca_achieved_gbs']), 'GB/s', round(r['ca_roofline_frac'], 4), 'env-steps/s %.3g' % r['env_steps_per_s'])
" 2> gpurun_out/abw_$V.err || exit 1
done
