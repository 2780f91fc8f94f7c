"""Golden vectors for the spectral diagnostics, made by the REFERENCE's
own functions (this container only: /root/reference does not exist on the GPU box).

Imported from the reference (read-only, never copied):
  model/fmSupportLib.py  estimatePSD (:66-140), DFT (:46-60)
Inputs: an FM-demodulated synthetic broadcast (the oracle front end on rtsdr.synth IQ, the
signal the reference plots at 240 kS/s), a tone-plus-noise record, and random vectors for
the DFT.  Cases cover ragged lengths (a partial last segment), NFFT 2..4096, and n < NFFT
(no segments: the reference returns 0/0 = NaN).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_psd_golden.py
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, "/root/reference/model")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

from fmSupportLib import DFT, estimatePSD  # noqa: E402  (reference)

import fm_oracle  # noqa: E402
import rtsdr  # noqa: E402  (only for the synthetic IQ generator)

PSD_CASES = [("demod", 512, 240e3, 512 * 9 + 123), ("demod", 4096, 240e3, 4096 * 3),
             ("demod", 64, 240e3, 1000), ("tone", 256, 48e3, 256 * 5), ("tone", 2, 48e3, 7),
             ("tone", 1024, 48e3, 1000)]
DFT_SIZES = [1, 2, 37, 256, 1000]


def signals():
    iq = rtsdr.synth.fm_iq(64_000, seed=21)
    b = fm_oracle.mono_coeffs(101)[0]
    i_f = fm_oracle.lfilter_fir(b, iq[0::2].astype(np.float64))[::10]
    q_f = fm_oracle.lfilter_fir(b, iq[1::2].astype(np.float64))[::10]
    demod, _ = fm_oracle.fm_demod_arctan(i_f, q_f, 0.0)
    rng = np.random.default_rng(4)
    t = np.arange(20_000) / 48e3
    tone = np.sin(2 * np.pi * 1e3 * t) + 0.3 * np.cos(2 * np.pi * 7.5e3 * t) + 0.01 * rng.standard_normal(len(t))
    # f32-representable samples: the GPU path may also take the pipeline's f32 buffers
    return {"demod": demod.astype(np.float32).astype(np.float64),
            "tone": tone.astype(np.float32).astype(np.float64)}


def main():
    sig = signals()
    out = {}
    for j, (name, nfft, fs, n) in enumerate(PSD_CASES):
        x = sig[name][:n]
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            f, p = estimatePSD(x, nfft, fs)
        fo, po = fm_oracle.estimate_psd(x, nfft, fs)
        assert np.array_equal(f, fo)
        assert np.array_equal(np.isnan(p), np.isnan(po)) and np.nanmax(np.abs(p - po), initial=0) < 1e-9, j
        out[f"psd{j}_x"], out[f"psd{j}_freq"], out[f"psd{j}_psd"] = x, f, p
        out[f"psd{j}_cfg"] = np.array([nfft, fs])
    rng = np.random.default_rng(9)
    for n in DFT_SIZES:
        x = rng.standard_normal(n)
        X = DFT(x)
        assert np.max(np.abs(X - fm_oracle.dft(x)), initial=0) < 1e-9 * max(1.0, np.max(np.abs(X)))
        out[f"dft{n}_x"], out[f"dft{n}_X"] = x, X
    np.savez_compressed(os.path.join(HERE, "psd.npz"), **out)
    print(f"{len(PSD_CASES)} PSD cases, {len(DFT_SIZES)} DFT sizes; restatement agrees")


if __name__ == "__main__":
    main()
