#!/bin/bash
# r02d: LDS row pitch A/B (CWP 320 vs 288), the C3/C4 value probe, and its PMC pass (clock + cycles).
set -u
mkdir -p gpurun_out/r02d
bash scripts/ab.sh base cwp288 base cwp288 > gpurun_out/r02d/ab.txt 2>&1 || exit 11
timeout -k 10 300 python scripts/c3c4_probe.py 20 > gpurun_out/r02d/c3c4.json 2> gpurun_out/r02d/c3c4.err || exit 12
R=$(pwd)
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_ANY SQ_WAIT_INST_ANY -d $R/gpurun_out/r02d/pmc_c3c4 -o run --output-format csv -- python3 $R/scripts/c3c4_probe.py 10 > $R/gpurun_out/r02d/pmc_c3c4.log 2>&1 || exit 13
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_WAVE_CYCLES -d $R/gpurun_out/r02d/pmc_lds -o run --output-format csv -- python3 $R/bench.py --no-cpu-baseline --headline-only --no-secondary --steps 4 --warmup 1 --reps 1 > $R/gpurun_out/r02d/pmc_lds.log 2>&1 || exit 14
echo done > $R/gpurun_out/r02d/done
