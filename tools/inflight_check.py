#!/usr/bin/env python3
"""Static check of hand-issued loads in flight: no instruction may read or write a register whose
VMEM load has not been retired by an s_waitcnt vmcnt.  Linear scan of one kernel's ISA (twice
over, so registers in flight across a loop's back edge are checked at the loop top too); FIFO of
outstanding VMEM instructions (loads return in order; stores only add to the count).  Only the
hand-issued loads (the `nt` loads of the inline-asm staging helpers) are tracked; the compiler's
own loads count toward vmcnt but are its business.
usage: python3 tools/inflight_check.py <file.s> <kernel-symbol-substring | --all>"""
import re
import sys

src, want = sys.argv[1], sys.argv[2]
text = open(src).read()
def regs(tok):
    """v12 / v[12:15] / a3 / a[0:3] -> {('v', 12), ...}"""
    out = set()
    for k, a, b in re.findall(r"\b([va])\[(\d+):(\d+)\]", tok):
        out |= {(k, i) for i in range(int(a), int(b) + 1)}
    for k, a in re.findall(r"\b([va])(\d+)\b", tok):
        out.add((k, int(a)))
    return out


VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")
def check(name, ins):
  queue = []           # [(index, dest regs)] oldest first
  bad = []
  for rnd in range(2):
      for i, l in enumerate(ins):
          op = l.split()[0]
          ops = l[len(op):]
          if op == "s_waitcnt":
              mv = re.search(r"vmcnt\((\d+)\)", ops)
              if mv:
                  n = int(mv.group(1))
                  while len(queue) > n:
                      queue.pop(0)
              continue
          touched = regs(ops)
          if VMEM.match(op):
              dest = set()
              if "load" in op and "_lds" not in op and ops.rstrip().endswith(" nt"):   # hand-issued (asm) loads
                  first = ops.split(",")[0]
                  dest = regs(first)
                  touched -= dest
              pending = set().union(*[q[1] for q in queue]) if queue else set()
              if touched & pending:
                  bad.append((rnd, i, l, sorted(touched & pending)[:4]))
              queue.append((i, dest))
              continue
          pending = set().union(*[q[1] for q in queue]) if queue else set()
          hit = touched & pending
          if hit:
              bad.append((rnd, i, l, sorted(hit)[:4]))
  print(f"{name[:90]}: {len(ins)} instructions, {len(bad)} touches of registers in flight")
  for rnd, i, l, h in bad[:40]:
      print(f"  pass {rnd} #{i}: {l}   {h}")
  return not bad


ok = True
names = re.findall(r"^(_Z\S*):", text, re.M) if want == "--all" else [n for n in re.findall(r"^(_Z\S*):", text, re.M) if want in n]
if not names:
    sys.exit(f"no symbol matching {want}")
for name in names:
    start = re.search(r"^" + re.escape(name) + r":", text, re.M).end()
    body = text[start:text.index(".Lfunc_end", start)]
    ins = [l.strip() for l in body.split("\n") if l.startswith("\t") and not l.strip().startswith((".", ";"))]
    ok &= check(name, ins)
sys.exit(0 if ok else 1)
