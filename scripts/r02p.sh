#!/bin/bash
# r02p: the observation kernels with extensions off (the plain-kernel path: base = adv_obs_plain_kernel, sel1 =
# adv_obs_sel_kernel, od1 = direct, os2048 = streaming) and the write-data probe (scripts/obs_data.py), two passes.
set -o pipefail
mkdir -p gpurun_out
V=gym-cellular-automata_amd/gymca_amd/_lib/variants
for pass in 1 2; do
  for X in ${VARIANTS:-base sel1}; do
    if [ $X = base ]; then L=""; else L=$V/$X.so; fi
    echo -n "$X "; GCA_LIB_PATH=$L timeout -k 10 120 python scripts/obs_data.py || exit 1
  done
done
