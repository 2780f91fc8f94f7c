#!/bin/bash
# A/B variant of libsdr.so (never shipped): one source recompiled with extra -D flags, the other
# objects taken from the product build (make -C real-time-software-defined-radio_amd/csrc first).
#   bash tools/ab_lib.sh <name> <source.hip> [-DFLAG=V ...]   -> real-time-software-defined-radio_amd/libsdr_<name>.so
#   then on the GPU box:  SDR_LIB=$GRAFT_REPO_ROOT/real-time-software-defined-radio_amd/libsdr_<name>.so python bench.py ...
set -e
name=$1; src=$2; shift 2
cd "$(dirname "$0")/../real-time-software-defined-radio_amd/csrc"
O=../_build_ab_$name
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-inline-asm \
  -Rpass-analysis=kernel-resource-usage "$@" -c "$src" -o $O/${src%.hip}.o 2> $O/${src%.hip}.res
python3 ../../tools/kres_gate.py $O/${src%.hip}.res
objs=""
for o in fe fe_mfma fir pll psd rx capi; do
  if [ "$o.hip" = "$src" ]; then objs="$objs $O/$o.o"; else objs="$objs ../_build/$o.o"; fi
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libsdr_$name.so $objs
echo "built libsdr_$name.so"
