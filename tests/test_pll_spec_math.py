"""CPU check of the method behind pll_spec_kernel (csrc/pll.hip): guess each step's wrap
integer from warm-up runs, solve the loop's linear form by a scan over chunks, check the
integers against the true step.  numpy restatement (vectorised over chunks) against the
sequential fract-form recurrence on the golden stereo pilot and RDS carrier inputs."""
import math
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def consts(freq, fs=240e3, bw=0.01):
    Kp, Ki = bw * 2.666, bw * bw * 3.555
    return dict(kA=2 * math.pi * Ki, kB=math.pi * Ki, kC=2 * math.pi * (Kp + Ki), kD=math.pi * (Kp + Ki),
                a=1 / (2 * math.pi), w=2 * math.pi * freq / fs)


def sequential(c, p, V, K):
    """Phases and V = integ - pi (Kp+Ki) after each step (the fast step of pll.hip)."""
    ph = np.empty(len(c))
    vs = np.empty(len(c))
    for k, ck in enumerate(c):
        t = ck - K["a"] * p
        f = t - math.floor(t)
        S = p + V
        V = K["kA"] * f + (V - K["kB"])
        p = K["kC"] * f + S
        ph[k] = p
        vs[k] = V
    return ph, vs


def solve(c, p0, V0, K, T, W, rounds=3):
    """(phases, rounds used) or (None, rounds) when the check never passes."""
    n = len(c)
    L = -(-n // T)
    TE = -(-n // L)
    C = np.concatenate([c, np.full(TE * L - n, np.nan)]).reshape(TE, L)
    live = ~np.isnan(C)

    def run(p, V, cols):
        fl = np.zeros(cols.shape)
        ph = np.zeros(cols.shape)
        for i in range(cols.shape[1]):
            col = cols[:, i]
            ok = ~np.isnan(col)
            t = col - K["a"] * p
            m = np.floor(t)
            f = t - m
            fl[:, i] = m
            S = p + V
            V = np.where(ok, K["kA"] * f + (V - K["kB"]), V)
            p = np.where(ok, K["kC"] * f + S, p)
            ph[:, i] = p
        return fl, ph, p, V

    ks = np.arange(TE)[:, None] * L - W + np.arange(W)[None, :]
    warm = np.where(ks >= 0, np.concatenate([c, [np.nan]])[np.clip(ks, 0, n)], np.nan)
    _, _, p, V = run(np.full(TE, p0), np.full(TE, V0), warm)
    fl, _, _, _ = run(p, V, C)
    A = np.array([[1 - K["kC"] * K["a"], 1.0], [-K["kA"] * K["a"], 1.0]])
    P = np.linalg.matrix_power(A, L)
    for r in range(rounds):
        z = np.zeros((TE, 2))
        for i in range(L):
            d = np.nan_to_num(C[:, i] - fl[:, i])
            zn = z @ A.T + np.stack([K["kC"] * d, K["kA"] * d - K["kB"]], 1)
            z = np.where(live[:, i:i + 1], zn, z)
        y = np.zeros((TE, 2))
        y[0] = (p0, V0)
        for j in range(TE - 1):
            y[j + 1] = P @ y[j] + z[j]
        fl2, ph, _, _ = run(y[:, 0], y[:, 1], C)
        miss = ((fl2 != fl) & live).any()
        fl = fl2
        if not miss:
            return ph.ravel()[:n], r + 1
    return None, rounds


@pytest.mark.parametrize("name,key,freq,T", [("mono_t151.npz", "bpf_recovery", 19e3, 256),
                                             ("rds_u8.npz", "pre_pll", 114e3, 512)])
def test_parallel_solve_matches_sequential(name, key, freq, T):
    x = np.load(os.path.join(G, name))[key].ravel().astype(np.float64)
    K = consts(freq)
    k = np.arange(len(x))
    c = ((np.where(x > 0, 0.0, math.pi)) - K["w"] * k) / (2 * math.pi) + 0.5
    ph, vs = sequential(c, 0.0, -K["kD"], K)
    B = 5120
    # blocks after the stream start (the acquisition block is the sequential kernel's case);
    # the kernel runs a block's sample 0 literally and solves samples 1..B-1 from that state
    for b0 in range(B, len(x) - B + 1, B):
        got, rounds = solve(c[b0 + 1:b0 + B], ph[b0], vs[b0], K, T, 256)
        assert got is not None, b0
        assert rounds == 1, (b0, rounds)
        assert np.abs(got - ph[b0 + 1:b0 + B]).max() < 1e-9, b0
