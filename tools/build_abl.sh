# Ablation builds of the u8 MFMA mono kernel (never shipped): libsdr_abl<mask>.so for each mask
# (fe_mfma.hip's SDR_FE_MFMA_ABL bits), the other objects taken from the product build.
#   bash tools/build_abl.sh 1 2 4 8 16   then   SDR_LIB=.../libsdr_abl<mask>.so python bench.py --iq u8 ...
set -e
cd "$(dirname "$0")/../real-time-software-defined-radio_amd/csrc"
for m in "$@"; do
  O=../_build_abl$m
  mkdir -p $O
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-function -Wno-inline-asm \
    -DSDR_FE_MFMA_ABL=$m -c fe_mfma.hip -o $O/fe_mfma.o &
done
wait
for m in "$@"; do
  O=../_build_abl$m
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o ../libsdr_abl$m.so $O/fe_mfma.o \
    ../_build/fe.o ../_build/fir.o ../_build/pll.o ../_build/psd.o ../_build/rx.o ../_build/capi.o
done
