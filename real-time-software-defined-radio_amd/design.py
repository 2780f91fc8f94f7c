"""Filter-coefficient design (host side, once per configuration).

The reference designs taps on the host too -- ``scipy.signal.firwin`` in the Python
model (model/fmMonoBlock.py:43,45,115,150,159; model/fmRDSblock.py:64-111) and
``impulseResponseLPF/BPF/RRC`` in the C++ (src/filter.cpp:19-93), the latter
recomputed every block (src/fm_radio.cpp:75).  Taps are data to the kernels; this
module only produces them.  Constants follow model/fmMonoBlock.py:22-32 and
model/fmRDSblock.py:24-47.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import signal

# model/fmMonoBlock.py:22-32
RF_FS = 2.4e6
RF_FC = 100e3
RF_TAPS = 151
RF_DECIM = 10
AUDIO_FS = 240e3
AUDIO_FC = 16e3
AUDIO_TAPS = 151
AUDIO_DECIM = 5

# model/fmRDSblock.py:38-47, 94-111
RDS_BPF = (54000.0, 60000.0)
RDS_SQ_BPF = (113500.0, 114500.0)
RDS_PLL_FREQ = 114000.0
RDS_PHASE_ADJ = math.pi / 3.3 - math.pi / 1.5
RDS_PLL_BW = 0.001
RDS_PLL_SCALE = 0.5
RDS_LPF_FC = 3000.0
RDS_UP, RDS_DOWN = 19, 80
RRC_FS = 57000.0
RRC_TAPS = 151

# stereo (model/fmMonoBlock.py:115-162)
PILOT_BPF = (18.5e3, 19.5e3)
STEREO_BPF = (22e3, 54e3)
PILOT_FREQ = 19e3
STEREO_PLL_SCALE = 2.0


def firwin_lpf(taps: int, fc: float, fs: float) -> np.ndarray:
    """signal.firwin(taps, fc/(fs/2), window='hann') as at model/fmMonoBlock.py:43."""
    return signal.firwin(taps, fc / (fs / 2), window=("hann"))


def firwin_bpf(taps: int, f_lo: float, f_hi: float, fs: float) -> np.ndarray:
    """signal.firwin(..., pass_zero='bandpass') as at model/fmMonoBlock.py:115."""
    return signal.firwin(taps, [f_lo / (fs / 2), f_hi / (fs / 2)], window=("hann"), pass_zero="bandpass")


def my_filterImpulseResponse(Fc, Fs, N_taps) -> np.ndarray:
    """Windowed sinc with a sin^2 window (model/fmSupportLib.py:144-154)."""
    fc = Fc / (Fs / 2)
    i = np.arange(N_taps, dtype=np.float64)
    off = i - (N_taps - 1) / 2
    arg = np.pi * fc * off
    with np.errstate(invalid="ignore", divide="ignore"):
        sinc = np.where(off == 0, fc, fc * np.sin(arg) / arg)
    return sinc * np.sin(np.pi * i / N_taps) ** 2


def impulseResponseRootRaisedCosine(Fs, N_taps) -> np.ndarray:
    """Root-raised-cosine taps, roll-off 0.90 at 2375 symbols/s (model/fmRRC.py:12-47).

    Same three cases as the reference: t == 0, |t| == Ts/(4 beta) (exact float
    comparison), and the general closed form; 1/Ts scale ignored as there.
    """
    ts, beta = 1 / 2375.0, 0.90
    t = (np.arange(N_taps, dtype=np.float64) - N_taps / 2) / Fs
    x = 4 * beta * t / ts
    with np.errstate(invalid="ignore", divide="ignore"):
        general = (np.sin(np.pi * t * (1 - beta) / ts) + x * np.cos(np.pi * t * (1 + beta) / ts)) / \
                  (np.pi * t * (1 - x * x) / ts)
    at_zero = 1.0 + beta * (4 / np.pi - 1)
    q = np.pi / (4 * beta)
    at_edge = beta / np.sqrt(2) * ((1 + 2 / np.pi) * np.sin(q) + (1 - 2 / np.pi) * np.cos(q))
    edge = (t == ts / (4 * beta)) | (t == -ts / (4 * beta))
    return np.where(t == 0.0, at_zero, np.where(edge, at_edge, general))


def mono_coeffs(rf_taps: int = RF_TAPS, audio_taps: int = AUDIO_TAPS):
    """(rf_coeff, audio_coeff) exactly as model/fmMonoBlock.py:43-45."""
    return firwin_lpf(rf_taps, RF_FC, RF_FS), firwin_lpf(audio_taps, AUDIO_FC, AUDIO_FS)


def stereo_coeffs(taps: int = RF_TAPS):
    """(pilot BPF, stereo-band BPF, stereo LPF), model/fmMonoBlock.py:115,150,159."""
    return (firwin_bpf(taps, *PILOT_BPF, AUDIO_FS),
            firwin_bpf(taps, *STEREO_BPF, AUDIO_FS),
            firwin_lpf(taps, 16e3, AUDIO_FS))


def rds_coeffs(taps: int = RF_TAPS):
    """RDS filters of model/fmRDSblock.py:88-111 (extract, squared BPF, 3k LPF, anti-image, RRC)."""
    return dict(
        extract=firwin_bpf(taps, *RDS_BPF, AUDIO_FS),
        square=firwin_bpf(taps, *RDS_SQ_BPF, AUDIO_FS),
        lpf=firwin_lpf(taps, RDS_LPF_FC, AUDIO_FS),
        anti_img=signal.firwin(taps, (57000 / 2) / ((240000 * 19) / 2), window=("hann")),
        rrc=impulseResponseRootRaisedCosine(RRC_FS, RRC_TAPS),
    )
