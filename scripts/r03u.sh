#!/bin/bash
# kernel trace of the Windy env step, fused vs three-kernel, 256^2 and 512^2 (1024 envs)
R=$(pwd)
O=$R/gpurun_out/r03u
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
for cfg in "256 1024 100 1" "256 1024 100 0" "512 1024 100 1" "512 1024 100 0"; do
  N=$(echo $cfg | tr ' ' '_')
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/tr_$N -o run --output-format csv -- python3 $R/scripts/windy_env_profile.py $cfg > $O/tr_$N.log 2>&1 || exit 1
done
echo done > $O/done.txt
