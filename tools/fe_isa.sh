#!/bin/bash
# usage: tools/fe_isa.sh <symbol-substring>...   (compiles tools/fe_tune.hip, prints ISA mix + regs)
cd /root/repo
out=$(hipcc --offload-arch=gfx950 -O3 -std=c++17 tools/fe_tune.hip -o tools/fe_tune -save-temps 2>&1 | grep -E "error" | head -5)
if [ -n "$out" ]; then echo "$out"; rm -f fe_tune-hip-* fe_tune-host-*; exit 1; fi
S=fe_tune-hip-amdgcn-amd-amdhsa-gfx950.s
for v in "$@"; do
  python3 tools/isa_mix.py $S "$v" 14
  grep -A30 "\.name:.*$v" $S | grep -E "vgpr_count|sgpr_count|spill|agpr" | tr '\n' ' '; echo
done
cp $S /tmp/last_fe_tune.s
rm -f fe_tune-hip-* fe_tune-host-*
