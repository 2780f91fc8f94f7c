"""How far a locked fmPll stays from its wrap: distance of fract(t_k) from 0 / 1 along the
golden stereo pilot (tests/golden/mono_t151.npz bpf_recovery) and RDS carrier
(rds_u8.npz pre_pll) inputs, fract-form step of csrc/pll.hip.  The parallel solve
(pll_spec_kernel) guesses each step's integer part from a warm-up run; a margin far above
rounding is what makes that guess robust.  CPU only; prints one line per input."""
import math, os
import numpy as np

G = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden")


def margins(x, freq, fs=240e3, bw=0.01):
    Kp, Ki = bw * 2.666, bw * bw * 3.555
    kA, kB, kC, kD = 2 * math.pi * Ki, math.pi * Ki, 2 * math.pi * (Kp + Ki), math.pi * (Kp + Ki)
    w = 2 * math.pi * freq / fs
    p, V = 0.0, -kD
    dist = np.empty(len(x))
    for k, xk in enumerate(x):
        c = ((0.0 if xk > 0 else math.pi) - w * k) / (2 * math.pi) + 0.5
        t = c - p / (2 * math.pi)
        f = t - math.floor(t)
        dist[k] = min(f, 1 - f)
        S = p + V
        V = kA * f + (V - kB)
        p = kC * f + S
    return dist


if __name__ == "__main__":
    mono = np.load(os.path.join(G, "mono_t151.npz"))
    rds = np.load(os.path.join(G, "rds_u8.npz"))
    for name, x, f in (("stereo pilot", mono["bpf_recovery"].ravel(), 19e3), ("RDS carrier", rds["pre_pll"].ravel(), 114e3)):
        d = margins(x, f)
        print(f"{name}: {len(x)} steps, min distance from the wrap {d[1:].min():.4f} "
              f"(steps 1-2000), {d[2000:].min():.4f} (after 2000)")
