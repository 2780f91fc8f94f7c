"""Golden vectors for the mode-1 audio resampler, made by the REFERENCE's
own C++ (this container only: /root/reference does not exist on the GPU box).

  * `make -C oracle ref` compiles /root/reference/src/filter.cpp where it lies into
    oracle/_ref/libref_fe.so together with oracle/ref_driver.cpp, whose
    ref_mode1_resample_blocks runs convolveWithDecimMode1 (src/filter.cpp:222-259) block by
    block as src/fm_radio.cpp:228 does (output zeroed between blocks, :305; its raw-history
    zi carried).
  * Input: the 250 kS/s IF of a synthetic 2.5 MS/s FM broadcast (the oracle front end:
    151-tap firwin LPF at 100 kHz, decimate by 10, atan2 demod), 4 blocks of 15 360 samples
    (307 200-byte u8 blocks / 20, src/fm_radio.cpp:23, :228).
  * Filter: 24/125 at 6 MHz, 16 kHz cutoff.  The reference designs 151*24 = 3624 taps with
    its sinc formula (src/fm_radio.cpp:176-179, :200; src/filter.cpp:19-38), which puts
    0/0 = NaN at tap 1812 for an even count, so its mode-1 audio is NaN (written as 0 at
    :290-293).  The pin uses a NaN-free 3 623-tap firwin (hann) design passed to the same
    reference code.
Stored: x, taps, and the reference's y (floor(15360*24/125) = 2 949 outputs per block).

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_mode1_golden.py
"""
from __future__ import annotations

import ctypes
import os
import subprocess
import sys

import numpy as np
from scipy import signal

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.dont_write_bytecode = True
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "oracle"))

import fm_oracle  # noqa: E402
import rtsdr  # noqa: E402  (only for the synthetic IQ generator)

BLOCK, NBLOCKS, UP, DOWN, TAPS = 15_360, 4, 24, 125, 3623


def if_signal():
    fs = 2.5e6
    iq = rtsdr.synth.fm_iq(BLOCK * NBLOCKS * 10, seed=31, fs=fs)
    b = signal.firwin(151, 100e3 / (fs / 2), window="hann")
    i_f = fm_oracle.lfilter_fir(b, iq[0::2].astype(np.float64))[::10]
    q_f = fm_oracle.lfilter_fir(b, iq[1::2].astype(np.float64))[::10]
    demod, _ = fm_oracle.fm_demod_arctan(i_f, q_f, 0.0)
    return demod.astype(np.float32)


def main():
    subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "ref"], check=True, capture_output=True)
    lib = ctypes.CDLL(os.path.join(REPO, "oracle", "_ref", "libref_fe.so"))
    fn = lib.ref_mode1_resample_blocks
    fp = ctypes.POINTER(ctypes.c_float)
    fn.argtypes = [fp, ctypes.c_int64, ctypes.c_int64, fp, ctypes.c_int, ctypes.c_int, ctypes.c_int, fp]
    fn.restype = None
    x = if_signal()
    taps = signal.firwin(TAPS, 16e3 / (6e6 / 2), window="hann")
    h32 = taps.astype(np.float32)
    ny = BLOCK * UP // DOWN
    y = np.zeros(NBLOCKS * ny, dtype=np.float32)
    fn(x.ctypes.data_as(fp), NBLOCKS, BLOCK, h32.ctypes.data_as(fp), TAPS, DOWN, UP, y.ctypes.data_as(fp))
    # the restatement (lfilter on the zero-stuffed stream, [::down], * up) on the same f32 taps
    zi = np.zeros(TAPS - 1)
    worst = 0.0
    for b in range(NBLOCKS):
        yo, zi = fm_oracle.resample(x[b * BLOCK:(b + 1) * BLOCK].astype(np.float64), h32.astype(np.float64),
                                    zi, UP, DOWN)
        first = 0 if b == 0 else -(-(TAPS - 1) // DOWN)
        d = np.abs(yo[first:ny] / UP - y[b * ny + first:(b + 1) * ny])
        worst = max(worst, float(d.max()))
    assert worst < 1e-5, worst
    np.savez_compressed(os.path.join(HERE, "mode1.npz"), x=x, taps=h32, y=y, block=BLOCK, up=UP, down=DOWN)
    print(f"mode-1 resampler: {NBLOCKS} blocks x {ny} outputs; restatement within {worst:.2e} of the reference")


if __name__ == "__main__":
    main()
