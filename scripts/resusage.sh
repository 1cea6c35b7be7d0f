#!/bin/bash
# Print VGPRs / scratch / occupancy per kernel of one HIP source (gfx950).
# Usage: bash scripts/resusage.sh gym-cellular-automata_amd/csrc/gca_alex.hip [name-filter]
f=$1; filt=${2:-.}
hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -ffp-contract=off -munsafe-fp-atomics -c "$f" -o /dev/null \
  -Rpass-analysis=kernel-resource-usage 2>&1 | grep -E "Function Name|VGPRs:|ScratchSize|Occupancy" | \
  sed -E 's/.*remark: +//; s/ \[-Rpass.*//' | paste - - - - | grep -E "$filt" | \
  sed -E 's/Function Name: _ZN12_GLOBAL__N_1[0-9]+//; s/EEEv.*\tVGPRs/ VGPRs/; s/\t/ /g'
