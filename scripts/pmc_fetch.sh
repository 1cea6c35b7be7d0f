#!/bin/bash
# FETCH_SIZE / WRITE_SIZE per alex_step launch for library variants: bash scripts/pmc_fetch.sh <variant|base>...
# (headline loop only; one rocprofv3 --pmc pass per counter group and variant)
R=${GRAFT_REPO_ROOT:-$(pwd)}
mkdir -p $R/gpurun_out
cd /tmp && export TMPDIR=/tmp
for V in "$@"; do
  if [ "$V" = base ]; then L=""; else L=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants/$V.so; fi
  for C in FETCH_SIZE WRITE_SIZE; do
    GCA_LIB_PATH=$L timeout -s KILL 120 rocprofv3 --pmc $C -d $R/gpurun_out/pmcf_${V}_$C -o run --output-format csv -- \
      python3 $R/bench.py --no-cpu-baseline --headline-only --no-secondary --steps 4 --warmup 1 > $R/gpurun_out/pmcf_${V}_$C.log 2>&1 || exit 1
    python3 - "$R/gpurun_out/pmcf_${V}_$C" "$V" "$C" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
v = [float(r["Counter_Value"]) for r in csv.DictReader(open(f)) if "alex_step" in r["Kernel_Name"]]
m = sum(v) / len(v)
cells = 4096 * 65536
k = 2 if sys.argv[3] == "FETCH_SIZE" else 1
print(sys.argv[2], sys.argv[3], "per launch KB", round(m), "-> B/cell", round(k * m * 1024 / cells, 3))
PY
  done
done
