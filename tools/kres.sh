#!/bin/bash
# Per-kernel VGPR / scratch / occupancy summary of a HIP source: tools/kres.sh file.hip [filter]
f=$1; pat=${2:-.}
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=fast -munsafe-fp-atomics -c $f -o /tmp/kres.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  awk '/Function Name:/{name=$NF} /VGPRs:/{v=$NF} /AGPRs:/{ag=$NF} /ScratchSize/{sc=$NF} /Occupancy/{oc=$NF; print name, "vgpr="v, "agpr="ag, "scratch="sc, "occ="oc}' | grep -- "$pat" | sed 's/\[-Rpass-analysis=kernel-resource-usage\]//g'
