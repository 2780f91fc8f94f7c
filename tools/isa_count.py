#!/usr/bin/env python3
"""Instruction mix of one kernel in a hipcc -save-temps .s file (tuning aid).
usage: isa_count.py FILE.s SUBSTRING [SUBSTRING...]"""
import collections
import re
import sys

src = open(sys.argv[1]).read()
funcs = re.findall(r"^([_A-Za-z][^\s:]*):[^\n]*\n(.*?)^\.Lfunc_end\d+:", src, re.S | re.M)
for key in sys.argv[2:]:
    for name, body in funcs:
        if key not in name:
            continue
        ins = [l.split()[0] for l in body.split('\n')
               if l.startswith('\t') and not l.startswith(('\t.', '\t;')) and l.strip()]
        c = collections.Counter(ins)
        tot = len(ins)
        grp = lambda pre: sum(v for k, v in c.items() if k.startswith(pre))
        print(f"{name[:90]}\n  total {tot}  valu {grp('v_')}  salu {grp('s_')}  ds {grp('ds_')}  "
              f"vmem {grp('global_') + grp('buffer_')}  accvgpr {sum(v for k, v in c.items() if 'accvgpr' in k)}  "
              f"pk_fma {c['v_pk_fma_f32']}  cndmask {c['v_cndmask_b32_e32'] + c['v_cndmask_b32_e64']}  "
              f"scratch {grp('scratch_')}  waitcnt {c['s_waitcnt']}  branch {grp('s_cbranch')}")
