# Diagnostic build of libsdr (never shipped): libsdr_<name>.so with the given -D flags, e.g.
#   bash tools/build_dbg.sh dbg -DSDR_PLL_SPEC_PROF
# then run a script with SDR_LIB=real-time-software-defined-radio_amd/libsdr_dbg.so.
set -e
NAME=$1
shift
cd "$(dirname "$0")/../real-time-software-defined-radio_amd/csrc"
O=../_build_$NAME
mkdir -p $O
for f in fe fe_mfma fir pll psd rx capi; do
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-inline-asm "$@" -c $f.hip -o $O/$f.o &
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libsdr_$NAME.so $O/*.o
