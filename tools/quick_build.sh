#!/bin/bash
# Tuning build: kron_v5 source $1 compiled with -DPOMS_V5_QUICK (p = 3 production
# kernels only), linked with the other objects of poms_amd/_obj into $2.
# Run with POMS_HIP_LIB=$2; never replaces poms_amd/libpoms_hip.so.
set -eu
ROOT=$(cd "$(dirname "$0")/.." && pwd)
SRC=$1; OUT=$2
T=$(mktemp -d)
cp "$SRC" $T/kron_v5.hip
cp "$ROOT/poms_amd/csrc/common.hpp" $T/
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fPIC -std=c++17 -Wall -Wno-unused-function -munsafe-fp-atomics \
    -DPOMS_V5_QUICK -I "$ROOT/include" -c $T/kron_v5.hip -o $T/kron_v5.o
objs=""
for s in kron_fused kron_dpp kron_v4 vec_ops transfer kron_solve stencil_general comm poms_abi; do
  objs="$objs $ROOT/poms_amd/_obj/$s.hip.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$OUT" $T/kron_v5.o $objs -L/opt/rocm/lib -lrccl
rm -rf $T
echo "built $OUT"
