#!/bin/bash
# GPU session (r05): the GPU suite, the fused-frame A/B (in-tree library vs variants built by scripts/build_variant.sh),
# a PMC profile of the fused-frame marching step, and the bench. Each step time-limited; a crash / abort / time limit
# ends the session. Usage (GPU box, repo root): bash scripts/gpu_frame_ab.sh <tag> "<variants>" [bench: 1|0]
TAG=$1; VARS=$2; BENCH=${3:-1}
R=$(pwd)
V=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
O=$R/gpurun_out/$TAG
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_gpu.log 2>&1
RC=$?; echo "pytest exit $RC" >> $O/pytest_gpu.log
[ $RC -eq 0 ] || [ $RC -eq 1 ] || exit 20
for pass in 1 2 3; do
  echo "pass $pass main $(timeout -k 10 180 python3 -u scripts/ab_march.py --only march ${AB_ARGS:---rgb-only} --reps 5)" >> $O/ab.txt || exit 21
  for v in $VARS; do
    echo "pass $pass $v $(GCA_LIB_PATH=$V/$v.so timeout -k 10 180 python3 -u scripts/ab_march.py --only march ${AB_ARGS:---rgb-only} --reps 5)" >> $O/ab.txt || exit 22
  done
done
P=$O/prof_rgb
mkdir -p $P
cd /tmp && export TMPDIR=/tmp
A="$R/scripts/ab_march.py --only march --rgb-only --reps 2"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $P/trace -o run --output-format csv -- python3 $A > $P/trace.log 2>&1 || exit 23
for PASS in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" "SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU"; do
  N=$(echo $PASS | tr ' ' '_' | cut -c1-40)
  timeout -k 10 300 rocprofv3 --pmc $PASS -d $P/pmc_$N -o run --output-format csv -- python3 $A > $P/pmc_$N.log 2>&1 || echo "pmc pass $PASS failed: $?" >> $P/errors.txt
done
echo profile done > $P/done.txt
cd $R
if [ "$BENCH" = "1" ]; then timeout -k 10 600 python bench.py > $O/bench.json 2> $O/bench.err || exit 26; fi
echo done > $O/done.txt
