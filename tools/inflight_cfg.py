#!/usr/bin/env python3
"""Path-sensitive form of tools/inflight_check.py: the same rule (no instruction may read or
write a register whose hand-issued `nt` VMEM load has not been retired by an s_waitcnt vmcnt),
checked over the kernel's control-flow graph instead of its linear layout.  The state carried
along a path is the FIFO of outstanding VMEM instructions (hand-issued loads with their
destination registers, everything else as an empty entry); every (block, state) pair reachable
from the entry is visited once.  A layout in which a block reached only with nothing in flight
sits after a load in the text is a false positive of the linear check and passes here.
usage: python3 tools/inflight_cfg.py <file.s> <kernel-symbol-substring | --all>"""
import re
import sys

VMEM = re.compile(r"^(global_|buffer_|flat_|scratch_)")


def regs(tok):
    out = set()
    for k, a, b in re.findall(r"\b([va])\[(\d+):(\d+)\]", tok):
        out |= {(k, i) for i in range(int(a), int(b) + 1)}
    for k, a in re.findall(r"\b([va])(\d+)\b", tok):
        out.add((k, int(a)))
    return out


def blocks_of(body):
    """[(label, [instructions], [successor labels])] in layout order"""
    blocks, cur, lab = [], [], "entry"
    for raw in body.split("\n"):
        l = raw.strip()
        m = re.match(r"^(\.LBB\w+):", l) or re.match(r"^; (%bb\.\d+):", l)
        if m:
            blocks.append([lab, cur])
            lab, cur = m.group(1), []
            continue
        if raw.startswith("\t") and l and not l.startswith((".", ";")):
            cur.append(l)
    blocks.append([lab, cur])
    out = []
    for i, (lab, ins) in enumerate(blocks):
        nxt = blocks[i + 1][0] if i + 1 < len(blocks) else None
        succ, fall = [], True
        for l in ins:
            op = l.split()[0]
            if op == "s_branch":
                succ.append(l.split()[1]); fall = False
            elif op.startswith("s_cbranch"):
                succ.append(l.split()[1])
            elif op in ("s_endpgm", "s_setpc_b64"):
                fall = False
        if fall and nxt is not None:
            succ.append(nxt)
        out.append((lab, ins, succ))
    return out


def check(name, body):
    bl = blocks_of(body)
    idx = {lab: i for i, (lab, _, _) in enumerate(bl)}
    seen, work, bad = set(), [(0, ())], []
    while work:
        b, state = work.pop()
        if (b, state) in seen:
            continue
        seen.add((b, state))
        lab, ins, succ = bl[b]
        q = list(state)
        for l in ins:
            op = l.split()[0]
            ops = l[len(op):]
            if op == "s_waitcnt":
                mv = re.search(r"vmcnt\((\d+)\)", ops)
                if mv:
                    n = int(mv.group(1))
                    while len(q) > n:
                        q.pop(0)
                continue
            touched = regs(ops)
            dest = frozenset()
            if VMEM.match(op) and "load" in op and "_lds" not in op and ops.rstrip().endswith(" nt"):
                dest = frozenset(regs(ops.split(",")[0]))
                touched -= dest
            pending = set().union(*q) if q else set()
            if touched & pending:
                bad.append((lab, l, sorted(touched & pending)[:4]))
            if VMEM.match(op):
                # entries past the largest count a wait here could name do not change the outcome
                q.append(dest)
                q = q[-64:]
        for s in succ:
            if s in idx:
                work.append((idx[s], tuple(q)))
    uniq = sorted(set((lab, l, tuple(h)) for lab, l, h in bad))
    print(f"{name[:90]}: {len(seen)} (block, state) pairs, {len(uniq)} touches of registers in flight")
    for lab, l, h in uniq[:40]:
        print(f"  {lab}: {l}   {list(h)}")
    return not uniq


text = open(sys.argv[1]).read()
want = sys.argv[2]
names = [n for n in re.findall(r"^(_Z\S*):", text, re.M) if want == "--all" or want in n]
if not names:
    sys.exit(f"no symbol matching {want}")
ok = True
for name in names:
    start = re.search(r"^" + re.escape(name) + r":", text, re.M).end()
    ok &= check(name, text[start:text.index(".Lfunc_end", start)])
sys.exit(0 if ok else 1)
