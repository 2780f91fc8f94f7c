"""fmPll through the parallel solve (pll_spec_kernel, csrc/pll.hip): the recurrence of a
block solved by chunk guesses + a scan of the loop's linear form, checked against the true
step, with the sequential kernel for whatever the check rejects.  Compared with the oracle's
restatement of model/fmPll.py:4-46 over chained blocks.  Run on an MI355X: pytest -m gpu."""
import numpy as np
import pytest

from conftest import maxabs

pytestmark = pytest.mark.gpu

FS = 240e3


def pilot(n, f0, seed, noise=0.05, phase=0.3):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    return (np.cos(2 * np.pi * f0 / FS * t + phase) + noise * rng.standard_normal(n)).astype(np.float32)


def chained(sdr, oracle, x, blocks, freq, scale, adj=0.0):
    st = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    sr = list(st)
    err = 0.0
    for a, b in blocks:
        nco, ncoq, st = sdr.fmPll(x[a:b], freq, FS, st, scale, adj)
        nr, nqr, sr = oracle.fm_pll(x[a:b].astype(np.float64), freq, FS, sr, scale, adj)
        err = max(err, maxabs(nco[1:], nr[1:]), maxabs(ncoq[1:], nqr[1:]))
        assert maxabs(st, sr) < 1e-6, (a, b)
    return err


@pytest.mark.parametrize("scale,adj", [(2.0, 0.0), (0.5, -np.pi / 3)])
def test_pll_locked_pilot_blocks(sdr, gpu_ctx, oracle, scale, adj):
    """C5-sized blocks (15 360 samples) of a slightly off-frequency pilot with noise: after the
    first block the loop is locked and the parallel solve completes every block; scale 0.5
    (RDS) makes a 2 pi slip of the phase estimate visible in the NCO."""
    B = 15360
    x = pilot(6 * B, 19e3 + 3.0, seed=11)
    err = chained(sdr, oracle, x, [(k * B, (k + 1) * B) for k in range(6)], 19e3, scale, adj)
    assert err < 2e-6


@pytest.mark.parametrize("n", [2, 3, 257, 5120, 16385, 16386])
def test_pll_block_sizes(sdr, gpu_ctx, oracle, n):
    """Block lengths around the solve's chunking (256 chunks, the last one short) and its
    16 385-sample limit (beyond it the sequential kernel runs)."""
    x = pilot(3 * n, 19e3, seed=n)
    err = chained(sdr, oracle, x, [(0, n), (n, 2 * n), (2 * n, 3 * n)], 19e3, 2.0)
    assert err < 2e-6


def test_pll_unlocked_input(sdr, gpu_ctx, oracle):
    """A weak pilot in noise at the start of a stream (acquisition): whatever the check
    rejects goes to the sequential kernel; results as the oracle's."""
    x = pilot(3 * 4000, 19e3 + 40.0, seed=3, noise=0.8)
    err = chained(sdr, oracle, x, [(0, 4000), (4000, 8000), (8000, 12000)], 19e3, 2.0)
    assert err < 2e-6
