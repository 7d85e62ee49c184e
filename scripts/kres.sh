#!/bin/bash
# Register / LDS / scratch use of the anomod kernels in one HIP source file.
# usage: scripts/kres.sh csrc/edge_agg.hip [extra hipcc flags]
src=$1; shift
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -munsafe-fp-atomics "$@" -c "$src" \
  -o /tmp/kres_$$.o -Rpass-analysis=kernel-resource-usage 2>&1 |
  grep -E "remark: (Function Name|    VGPRs:|    ScratchSize|    Occupancy|    LDS Size)" |
  sed -E 's/.*remark: *//; s/ \[-Rpass-analysis=kernel-resource-usage\]//' |
  paste - - - - - | grep "_ZN6anomod" | sed -E 's/Function Name: _ZN6anomod12_GLOBAL__N_1[0-9]+//'
rm -f /tmp/kres_$$.o
