"""RDS link layer (model/fmRDSblock.py:207-346).

The pin is tests/golden/rds_link.npz, written by make_rds_link_golden.py: the reference
script itself, run on synthetic IQ carrying coded RDS groups, printed its syndrome events,
and the oracle restatement reproduced them exactly.  Here:
  * the oracle against those events (CPU);
  * libsdr's C++ link layer (host code, no GPU) against the same events, symbols, bits and
    scanned bits, on the oracle's RRC input (CPU);
  * the whole RDS chain on the GPU (RdsBlockProcessor -> RdsLinkLayer) against the
    reference's events (gpu).
"""
import numpy as np
import pytest


def _split(z, key):
    parts, o = [], 0
    for n in z["n_" + key]:
        parts.append(z[key][o:o + n])
        o += n
    return parts


def _events(z):
    return [tuple(int(v) for v in e) for e in z["events"]]


def test_oracle_reproduces_reference_prints(oracle, golden):
    z = golden("rds_link.npz")
    link = oracle.rds_link(list(z["rrc_i"]))
    assert [e for r in link for e in r["events"]] == _events(z)
    assert sum(e[2] for e in _events(z)) >= 1          # the frame sync accepted syndromes


def test_cpp_link_layer_matches_reference(sdr, golden):
    z = golden("rds_link.npz")
    link = sdr.RdsLinkLayer()
    got = [link.process(x) for x in z["rrc_i"]]
    assert [e for r in got for e in r["events"]] == _events(z)
    for key in ("symbols", "bits", "diff"):
        for g, ref in zip((r[key] for r in got), _split(z, key)):
            np.testing.assert_array_equal(g, ref.astype(g.dtype))


def test_cpp_link_layer_block_size_invariance(sdr, golden, oracle):
    """Bits do not depend on how the RRC stream is cut into blocks of whole symbols."""
    z = golden("rds_link.npz")
    x = np.concatenate(list(z["rrc_i"]))
    a = sdr.RdsLinkLayer()
    whole = a.process(x)
    ref = oracle.rds_link([x])[0]
    assert whole["events"] == ref["events"]
    np.testing.assert_array_equal(whole["bits"], ref["bits"].astype(np.uint8))


def test_cpp_link_layer_rejects_short_blocks(sdr):
    link = sdr.RdsLinkLayer()
    with pytest.raises(Exception):
        link.process(np.zeros(10))


@pytest.mark.gpu
def test_gpu_rds_chain_to_frame_sync(sdr, gpu_ctx, golden):
    z = golden("rds_link.npz")
    iq = sdr.synth.fm_iq(int(z["n_complex"]), seed=int(z["seed"]), dtype=np.uint8, rds_groups=True)
    proc = sdr.RdsBlockProcessor(153_600)
    link = sdr.RdsLinkLayer()
    events = []
    nb = len(z["rrc_i"])
    for k in range(nb):
        out = proc.process(iq[2 * k * 153_600:2 * (k + 1) * 153_600])
        events += link.process(out["rrc_i"])["events"]
    assert events == _events(z)
