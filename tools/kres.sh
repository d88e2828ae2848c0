#!/bin/bash
# Per-kernel VGPR / spill / occupancy of dag_stem.hip (development helper).
# Usage: tools/kres.sh [extra hipcc flags...]
ROOT=$(cd "$(dirname "$0")/.." && pwd)
/opt/rocm/bin/hipcc -O3 -std=c++17 "$@" -I$ROOT/include -I$ROOT/stem_kernel_amd/csrc --offload-arch=gfx950 \
  -munsafe-fp-atomics -x hip -c $ROOT/stem_kernel_amd/csrc/kernels/dag_stem.hip -o /tmp/kres.o \
  -Rpass-analysis=kernel-resource-usage 2>&1 | sed 's/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  awk '/Function Name/ {n=$NF} /VGPRs:/ {v=$NF} /VGPRs Spill/ {sp=$NF} /Occupancy/ {print n, "vgpr=" v, "spill=" sp, "occ=" $NF}' |
  sed 's/_ZN2sk18sk_dag_stem_kernelILi\([0-9]*\)EEEvNS_10StemLaunchE/stem<\1>/'
