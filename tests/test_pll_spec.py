"""fmPll through the parallel solve (pll_spec_kernel, csrc/pll.hip): the recurrence of a
block solved by chunk guesses + a scan of the loop's linear form, checked against the true
step, with the sequential kernel for whatever the check rejects; and long calls (n > 16 385:
pseudo-blocks solved from warm-up guesses and chained).  Compared with the oracle's
restatement of model/fmPll.py:4-46 over chained blocks, and the solver counters
(sdr_pll_stats) asserted, so a solve that silently fell back to the sequential kernel fails
here.  Run on an MI355X: pytest -m gpu."""
import time

import numpy as np
import pytest

from conftest import long_blocks, maxabs

pytestmark = pytest.mark.gpu

FS = 240e3
NCO_TOL = 2e-6          # f32 NCO outputs vs the f64 oracle (3e-8 measured on locked blocks)


def pilot(n, f0, seed, noise=0.05, phase=0.3):
    rng = np.random.default_rng(seed)
    t = np.arange(n)
    return (np.cos(2 * np.pi * f0 / FS * t + phase) + noise * rng.standard_normal(n)).astype(np.float32)


@pytest.fixture(autouse=True)
def fresh_counters(gpu_ctx):
    gpu_ctx.pll_stats(reset=True)


def chained(sdr, oracle, x, blocks, freq, scale, adj=0.0, bw=0.01, times=None):
    st = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    sr = list(st)
    err = 0.0
    for a, b in blocks:
        t0 = time.perf_counter()
        nco, ncoq, st = sdr.fmPll(x[a:b], freq, FS, st, scale, adj, bw)
        if times is not None:
            times.append(time.perf_counter() - t0)
        nr, nqr, sr = oracle.fm_pll(x[a:b].astype(np.float64), freq, FS, sr, scale, adj, bw)
        err = max(err, maxabs(nco[1:], nr[1:]), maxabs(ncoq[1:], nqr[1:]))
        assert maxabs(st, sr) < 1e-6, (a, b)
    return err


def spec_total(s):
    return s["spec_r0"] + s["spec_r1"] + s["spec_r2"]


@pytest.mark.parametrize("scale,adj", [(2.0, 0.0), (0.5, -np.pi / 3)])
def test_pll_locked_pilot_blocks(sdr, gpu_ctx, oracle, scale, adj):
    """C5-sized blocks (15 360 samples) of a slightly off-frequency pilot with noise: after the
    first block the loop is locked and the parallel solve completes every block -- asserted on
    the solver counters, not only on the outputs; scale 0.5 (RDS) makes a 2 pi slip of the
    phase estimate visible in the NCO."""
    B = 15360
    x = pilot(6 * B, 19e3 + 3.0, seed=11)
    err = chained(sdr, oracle, x, [(k * B, (k + 1) * B) for k in range(6)], 19e3, scale, adj)
    assert err < NCO_TOL
    s = gpu_ctx.pll_stats()
    print("solver counters:", s)
    nb = long_blocks(B)                                        # pseudo-blocks per block
    assert s["recurrences"] == 6 * nb
    assert spec_total(s) >= 5 * nb and s["sequential"] <= nb, s   # every locked block in parallel
    assert s["spec_r0"] >= 5 * nb, s                              # ... in the first round


@pytest.mark.parametrize("n", [2, 3, 257, 5120, 16385, 16386, 3 * 16384 + 5])
def test_pll_block_sizes(sdr, gpu_ctx, oracle, n):
    """Block lengths around the solve's chunking (256 chunks, the last one short), its
    16 385-sample limit and the long-call split beyond it (16 386 = 2 pseudo-blocks of 8 193;
    3 x 16 384 + 5 = 4 pseudo-blocks of <= 14 336)."""
    x = pilot(3 * n, 19e3, seed=n)
    err = chained(sdr, oracle, x, [(0, n), (n, 2 * n), (2 * n, 3 * n)], 19e3, 2.0)
    assert err < NCO_TOL
    s = gpu_ctx.pll_stats()
    nb = long_blocks(n)
    assert s["recurrences"] == 3 * nb, s
    if n > 16385:
        assert s["long_guessed"] + s["long_chained"] == 3 * nb, s


def test_pll_unlocked_input(sdr, gpu_ctx, oracle):
    """A weak pilot in noise at the start of a stream (acquisition): whatever the check
    rejects goes to the sequential kernel; results as the oracle's."""
    x = pilot(3 * 4000, 19e3 + 40.0, seed=3, noise=0.8)
    err = chained(sdr, oracle, x, [(0, 4000), (4000, 8000), (8000, 12000)], 19e3, 2.0)
    assert err < NCO_TOL
    s = gpu_ctx.pll_stats()
    assert s["recurrences"] == 3 * long_blocks(4000)


@pytest.mark.parametrize("cfg", ["stereo", "rds"])
def test_pll_long_call_locked(sdr, gpu_ctx, oracle, cfg):
    """A device-resident span as ONE call: 8 x 15 360 samples (9 pseudo-blocks of 13 654) of a
    locked tone, then a second call continuing it.  Every pseudo-block must be solved in
    parallel (no sequential kernel): the stereo loop's pre-roll converges to 1e-9 and its blocks
    are accepted as guessed; the RDS loop (10x narrower) is fixed up from the chained start."""
    n = 8 * 15360
    if cfg == "stereo":
        x, freq, scale, adj, bw = pilot(2 * n, 19e3 + 1.0, seed=5), 19e3, 2.0, 0.0, 0.01
    else:
        x, freq, scale, adj, bw = pilot(2 * n, 114e3 - 5.7, seed=6, noise=0.02), 114e3, 0.5, np.pi / 3.3 - np.pi / 1.5, 0.001
    err = chained(sdr, oracle, x, [(0, n), (n, 2 * n)], freq, scale, adj, bw)
    assert err < NCO_TOL
    s = gpu_ctx.pll_stats()
    print(cfg, "solver counters:", s)
    nb = long_blocks(n)
    assert s["recurrences"] == 2 * nb, s
    assert s["long_guessed"] + s["long_chained"] == 2 * nb, s
    assert s["sequential"] <= 1, s                 # at most the acquisition block at the stream start
    assert s["long_maxgap"] <= 1e-9, s
    if cfg == "stereo":
        assert s["long_guessed"] >= 2 * nb - 2, s


def test_pll_long_call_zero_inputs(sdr, gpu_ctx, oracle):
    """Exact zeros inside a long call (the reference's atan2(-0*fQ, 0*fI) case): those
    pseudo-blocks go to the sequential kernel from their start; the chain still holds."""
    n = 4 * 16384
    x = pilot(n, 19e3, seed=9)
    x[20000:20010] = 0.0
    x[50000] = 0.0
    err = chained(sdr, oracle, x, [(0, n)], 19e3, 2.0)
    assert err < NCO_TOL
    s = gpu_ctx.pll_stats()
    assert s["recurrences"] == long_blocks(n) and s["sequential"] >= 2, s


@pytest.mark.parametrize("offset,noise", [(40.0, 0.8), (7.0, 0.3)])
def test_pll_long_call_unlocked(sdr, gpu_ctx, oracle, offset, noise):
    """Long calls on a loop that is NOT locked (a weak, 40 Hz-off pilot in heavy noise; a
    noisy 7 Hz offset): the pre-roll guesses are wrong, so the chain stops, hands pseudo-blocks
    their exact (chained) starts for re-solves in later rounds, and whatever the rounds leave
    runs sequentially from the chain's exact position.  Those hand-overs are the riskiest part
    of the long-call solver: NCO and carried state must still equal the oracle's (model/fmPll.py
    :4-46) over three chained calls, and the counters must show the non-trivial paths ran."""
    n = 4 * 16384 + 5
    x = pilot(3 * n, 19e3 + offset, seed=int(offset), noise=noise)
    times = []
    err = chained(sdr, oracle, x, [(0, n), (n, 2 * n), (2 * n, 3 * n)], 19e3, 2.0, times=times)
    assert err < NCO_TOL
    s = gpu_ctx.pll_stats()
    # the unlocked call's cost, host-to-host, for the record (the pseudo-blocks the chain hands to the one-thread
    # tail run serially, ~30 ns a step: the whole call fully serial would be ~2 ms of loop)
    print(f"offset {offset} noise {noise} call ms {[round(t * 1e3, 2) for t in times]} solver counters:", s)
    nb = long_blocks(n)
    assert s["recurrences"] == 3 * nb, s
    assert s["long_stops"] + s["long_tail"] + s["sequential"] + s["spec_r1"] + s["spec_r2"] > 0, s
    # (the call times are printed, not asserted: host wall-clock around host-device copies is not
    # a correctness property -- the solver counters above are the gate)
