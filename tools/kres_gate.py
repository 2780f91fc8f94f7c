#!/usr/bin/env python3
"""Build gate: every gfx950 kernel of libsdr must use no scratch memory.

The streaming FE kernels wait for their LDS-DMA and hand-issued LDS reads with counted
`s_waitcnt vmcnt(N)` / `lgkmcnt(N)` (csrc/fe.hip).  Those counts are exact only if the
compiler emits no memory operations of its own between them; a register spill to scratch
is exactly such an operation, and would make the kernel read stale LDS silently.  So the
build compiles every .hip with -Rpass-analysis=kernel-resource-usage (csrc/Makefile) and
this script fails the build if any kernel reports ScratchSize != 0 or dynamic stack use.

usage: kres_gate.py <remarks-file>...   (exit 1 with the offending kernels listed)
"""
import re
import sys


def parse(path):
    rows, cur = [], None
    with open(path, errors="replace") as f:
        for line in f:
            m = re.search(r"Function Name: (\S+)", line)
            if m:
                cur = {"name": m.group(1), "file": path}
                rows.append(cur)
                continue
            m = re.search(r"remark:\s+(ScratchSize \[bytes/lane\]|Dynamic Stack|VGPRs|AGPRs): (\S+)", line)
            if m and cur is not None:
                cur[m.group(1).split()[0]] = m.group(2)
    return rows


# Kernels allowed a bounded spill, each with the measurement that justifies it ("Build
# gate").  Only kernels without counted waits may appear here -- never the FE kernels.
ALLOW = {
    # (empty: r06's one entry -- the long-call solve's 20 B/lane with the compact rows' AF check
    # form -- went when its wave scans moved from ds_bpermute shuffles to DPP moves)
}


def main(paths):
    rows = [r for p in paths for r in parse(p)]
    if not rows:
        print("kres_gate: no kernel resource remarks found", file=sys.stderr)
        return 1

    def over(r):
        return int(r.get("ScratchSize", "0")) > ALLOW.get(r["name"], 0)
    bad = [r for r in rows if over(r) or r.get("Dynamic", "False") not in ("False", "0")]
    for r in bad:
        print(f"kres_gate: {r['name']} ({r['file']}): scratch {r.get('ScratchSize')} B/lane, "
              f"dynamic stack {r.get('Dynamic')}", file=sys.stderr)
    if bad:
        return 1
    allowed = [f"{r['name']} {r.get('ScratchSize')} B" for r in rows if r.get("ScratchSize", "0") != "0"]
    print(f"kres_gate: {len(rows)} kernels, no scratch" + (f" but the allowed {allowed}" if allowed else ""))
    return 0


if __name__ == "__main__":
    sys.exit(main(sys.argv[1:]))
