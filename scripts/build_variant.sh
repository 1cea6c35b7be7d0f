#!/bin/bash
# Build an A/B variant of libgca_hip.so (extra compiler flags, or another source tree via VARIANT_SRC) into
# gym-cellular-automata_amd/gymca_amd/_lib/variants/<name>.so; select it with GCA_LIB_PATH=<that path>.
# Usage: bash scripts/build_variant.sh <name> <flags...>
set -e
NAME=$1; shift
R=$(cd "$(dirname "$0")/.." && pwd)
C=${VARIANT_SRC:-$R/gym-cellular-automata_amd/csrc}  # VARIANT_SRC: another source tree (e.g. a git worktree)
O=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
B=$C/build/variant_$NAME
mkdir -p $O $B
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function -munsafe-fp-atomics $*"
for s in gca_util gca_windy gca_env gca_alex gca_alex_march gca_ds gca_obs gca_pine gca_init gca_bench; do
  /opt/rocm/bin/hipcc $F -c $C/$s.hip -o $B/$s.o &
done
wait
for s in gca_util gca_windy gca_env gca_alex gca_alex_march gca_ds gca_obs gca_pine gca_init gca_bench; do [ -f $B/$s.o ] || { echo "compile of $s failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $B/*.o -o $O/$NAME.so
echo $O/$NAME.so
