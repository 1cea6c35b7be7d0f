#!/bin/bash
# Like build_variant.sh, but recompiles ONE source with the extra flags and links it with the in-tree objects of the
# others (gym-cellular-automata_amd/csrc/build/*.o from `make`). Usage: bash scripts/build_variant1.sh <name> <src> <flags...>
set -e
NAME=$1; SRC=$2; shift 2
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/gym-cellular-automata_amd/csrc
O=$R/gym-cellular-automata_amd/gymca_amd/_lib/variants
B=$C/build/variant1_$NAME
mkdir -p $O $B
F="-O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -Wno-unused-function -munsafe-fp-atomics $*"
/opt/rocm/bin/hipcc $F -c $C/$SRC.hip -o $B/$SRC.o
OBJS="$B/$SRC.o $(ls $C/build/*.o | grep -v "/$SRC.o$")"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 $OBJS -o $O/$NAME.so
echo $O/$NAME.so
