"""Golden vectors for the RDS link layer, pinned by running the
REFERENCE script itself (this container only: /root/reference does not exist on the GPU box).

  1. Synthetic u8 IQ whose 57 kHz subcarrier carries coded RDS groups
     (rtsdr.synth.fm_iq(..., rds_groups=True)): 8 x 307 200 bytes, the slice
     model/fmRDSblock.py:60 keeps.
  2. model/fmRDSblock.py runs unmodified as __main__ in a scratch directory whose
     model/ entries are symlinks to /root/reference/model/*.py and whose
     data/samples_rds_1029.raw is the synthetic file (:57).  Its prints are the pin:
     'Initial offset for clock recovery', 'Start position', 'Syndrome X at position N'
     and 'False positive Syndrome X at position N' (:212, :249, :300-338).
  3. oracle/fm_oracle.py's rds_blocks + rds_link restatement must reproduce those
     prints exactly; its per-block RRC input, symbols, bits and syndrome events are
     stored in rds_link.npz together with the reference's events.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_rds_link_golden.py
"""
from __future__ import annotations

import os
import re
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_MODEL = "/root/reference/model"
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import fm_oracle  # noqa: E402
import rtsdr  # noqa: E402

SEED = 11
N_COMPLEX = 8 * 153_600
TYPES = {"A": 0, "B": 1, "C": 2, "D": 3}


def run_reference(iq_u8):
    with tempfile.TemporaryDirectory() as tmp:
        os.makedirs(os.path.join(tmp, "model"))
        os.makedirs(os.path.join(tmp, "data"))
        for f in os.listdir(REF_MODEL):
            if f.endswith(".py"):
                os.symlink(os.path.join(REF_MODEL, f), os.path.join(tmp, "model", f))
        iq_u8.tofile(os.path.join(tmp, "data", "samples_rds_1029.raw"))
        env = dict(os.environ, MPLBACKEND="Agg", PYTHONDONTWRITEBYTECODE="1")
        res = subprocess.run([sys.executable, "fmRDSblock.py"], cwd=os.path.join(tmp, "model"), env=env,
                             capture_output=True, text=True, timeout=1200)
        if res.returncode != 0:
            raise RuntimeError(res.stderr[-2000:])
        return res.stdout


def parse(stdout):
    events = []
    for line in stdout.splitlines():
        m = re.match(r"\s*(False positive )?Syndrome ([ABCD]) at position\s+(\d+)", line)
        if m:
            events.append((TYPES[m.group(2)], int(m.group(3)), 0 if m.group(1) else 1))
    offset = int(re.search(r"Initial offset for clock recovery\s+(\d+)", stdout).group(1))
    start = int(re.search(r"Start position\s+(\d+)", stdout).group(1))
    return events, offset, start


def main():
    iq = rtsdr.synth.fm_iq(N_COMPLEX, seed=SEED, dtype=np.uint8, rds_groups=True)
    stdout = run_reference(iq)
    ref_events, ref_offset, ref_start = parse(stdout)
    blocks = fm_oracle.rds_blocks(iq)
    link = fm_oracle.rds_link([b["rrc_i"] for b in blocks])
    events = [e for r in link for e in r["events"]]
    offset0 = int(np.where(blocks[0]["rrc_i"][0:24] == np.max(blocks[0]["rrc_i"][0:24]))[0][0])
    assert offset0 == ref_offset, (offset0, ref_offset)
    assert events == ref_events, (events[:10], ref_events[:10])
    accepted = sum(e[2] for e in events)
    print(f"reference: {len(ref_events)} syndrome prints ({accepted} in frame), offset {ref_offset}, "
          f"start {ref_start}; restatement identical")
    cat = lambda key, dt: np.concatenate([np.asarray(r[key], dtype=dt) for r in link])  # noqa: E731
    np.savez_compressed(
        os.path.join(HERE, "rds_link.npz"),
        seed=SEED, n_complex=N_COMPLEX,
        rrc_i=np.stack([b["rrc_i"] for b in blocks]),
        symbols=cat("symbols", np.float64), n_symbols=np.array([len(r["symbols"]) for r in link]),
        bits=cat("bits", np.uint8), n_bits=np.array([len(r["bits"]) for r in link]),
        diff=cat("diff", np.uint8), n_diff=np.array([len(r["diff"]) for r in link]),
        events=np.array(ref_events, dtype=np.int64).reshape(-1, 3),
        n_events=np.array([len(r["events"]) for r in link]),
        ref_offset=ref_offset, ref_start=ref_start)


if __name__ == "__main__":
    main()
