"""Generate the golden vectors in tests/golden/ by running the REFERENCE's own
functions (this container only: /root/reference does not exist on the GPU box).

Imported from the reference (read-only, never copied):
  model/fmSupportLib.py  fmDemodArctan, my_filterImpulseResponse, my_convoloution
  model/fmPll.py         fmPll
  model/fmRRC.py         impulseResponseRootRaisedCosine
plus scipy.signal.lfilter / firwin exactly as the reference calls them.  The loops
below follow model/fmMonoBlock.py:80-173 and model/fmRDSblock.py:127-204 statement by
statement, with three documented fixes:
  * fmMonoBlock.py:119 unpacks 2 of fmPll's 3 return values -> unpack 3;
  * fmMonoBlock.py:166-170 aliases the L/R arrays -> intended L=(a+s)/2, R=(a-s)/2;
  * fmPll.py:13 leaves ncoOutQ[0] uninitialised (np.empty) -> set to the carried
    quadrature value sin(theta_prev*scale+adj) (0 at stream start) before use.

Run:  PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import math
import os
import platform
import sys

import numpy as np
import scipy
from scipy import signal

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF_MODEL = "/root/reference/model"
sys.dont_write_bytecode = True
sys.path.insert(0, REF_MODEL)
sys.path.insert(0, REPO)

from fmPll import fmPll  # noqa: E402  (reference)
from fmRRC import impulseResponseRootRaisedCosine  # noqa: E402  (reference)
from fmSupportLib import fmDemodArctan, my_convoloution, my_filterImpulseResponse  # noqa: E402  (reference)

import rtsdr  # noqa: E402  (only for the synthetic IQ generator)


def ncoq0(state, freq, Fs, scale, adj):
    """Defined value for the reference's uninitialised ncoOutQ[0]."""
    off, phase = state[5], state[1]
    return math.sin((2 * math.pi * (freq / Fs) * off + phase) * scale + adj) if off > 0 else 0.0


def mono_loop(iq, block_size, rf_taps, stereo):
    """model/fmMonoBlock.py:43-173 with the reference's own functions."""
    rf_Fs, rf_Fc, rf_decim = 2.4e6, 100e3, 10
    audio_Fs, audio_Fc, audio_taps, audio_decim = 240e3, 16e3, 151, 5
    rf_coeff = signal.firwin(rf_taps, rf_Fc / (rf_Fs / 2), window=('hann'))
    audio_coeff = signal.firwin(audio_taps, audio_Fc / (audio_Fs / 2), window=('hann'))
    state_i = np.zeros(rf_taps - 1)
    state_q = np.zeros(rf_taps - 1)
    state_phase = 0
    state_recovery = np.zeros(151 - 1)
    state_extraction = np.zeros(151 - 1)
    audio_pre_state = np.zeros(audio_taps - 1)
    stereo_pre_state = np.zeros(151 - 1)
    recovery_state = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    res = {}
    block_count = 0
    while (block_count + 1) * block_size < len(iq):
        b0, b1 = block_count * block_size, (block_count + 1) * block_size
        i_filt, state_i = signal.lfilter(rf_coeff, 1.0, iq[b0:b1:2], zi=state_i)
        q_filt, state_q = signal.lfilter(rf_coeff, 1.0, iq[b0 + 1:b1:2], zi=state_q)
        i_ds = i_filt[::rf_decim]
        q_ds = q_filt[::rf_decim]
        fm_demod, state_phase = fmDemodArctan(i_ds, q_ds, state_phase)
        audio_filt, audio_pre_state = signal.lfilter(audio_coeff, 1.0, fm_demod, zi=audio_pre_state)
        audio_block = audio_filt[::audio_decim]
        r = dict(i_ds=i_ds, q_ds=q_ds, demod=fm_demod, audio=audio_block, phase=np.array([state_phase]),
                 zi_i=state_i.copy(), zi_q=state_q.copy(), audio_zi=audio_pre_state.copy())
        if stereo:
            bp_rec = signal.firwin(151, [18.5e3 / (audio_Fs / 2), 19.5e3 / (audio_Fs / 2)], window=('hann'),
                                   pass_zero="bandpass")
            bpf_recovery, state_recovery = signal.lfilter(bp_rec, 1.0, fm_demod, zi=state_recovery)
            recovery_pll, _, recovery_state = fmPll(bpf_recovery, 19e3, 240e3, recovery_state, 2)
            bp_ext = signal.firwin(151, [22e3 / (audio_Fs / 2), 54e3 / (audio_Fs / 2)], window=('hann'),
                                   pass_zero="bandpass")
            bpf_extraction, state_extraction = signal.lfilter(bp_ext, 1.0, fm_demod, zi=state_extraction)
            mixed = np.multiply(recovery_pll[0:len(bpf_extraction):1], bpf_extraction)
            mixed = mixed * 2
            stereo_coeff = signal.firwin(151, 16e3 / (audio_Fs / 2), window=('hann'))
            stereo_filt, stereo_pre_state = signal.lfilter(stereo_coeff, 1.0, mixed, zi=stereo_pre_state)
            stereo_block = stereo_filt[::5]
            r.update(bpf_recovery=bpf_recovery, nco=recovery_pll, bpf_extraction=bpf_extraction,
                     stereo=stereo_block, left=(audio_block + stereo_block) / 2,
                     right=(audio_block - stereo_block) / 2, pll_state=np.array(recovery_state, dtype=np.float64))
        for k, v in r.items():
            res.setdefault(k, []).append(np.asarray(v, dtype=np.float64))
        block_count += 1
    return {k: np.stack(v) for k, v in res.items()}


def rds_loop(iq_u8, block_size, nblocks_full):
    """model/fmRDSblock.py:57-204 with the reference's own functions."""
    rf_taps = 151
    iq_data = (iq_u8 - 128.0) / 128.0
    rf_coeff = signal.firwin(rf_taps, 100e3 / (2.4e6 / 2), window=('hann'))
    audio_Fs = 240000
    extract_RDS_coeff = signal.firwin(rf_taps, [54000 / (audio_Fs / 2), 60000 / (audio_Fs / 2)], window=('hann'),
                                      pass_zero="bandpass")
    square_coeff = signal.firwin(rf_taps, [113500 / (audio_Fs / 2), 114500 / (audio_Fs / 2)], window=('hann'),
                                 pass_zero="bandpass")
    phase_adj = math.pi / 3.3 - math.pi / 1.5
    lpf_coeff_rds = signal.firwin(rf_taps, 3000 / (audio_Fs / 2), window=('hann'))
    anti_img_coeff = signal.firwin(rf_taps, (57000 / 2) / ((240000 * 19) / 2), window=('hann'))
    rrc_coeff = impulseResponseRootRaisedCosine(57000, 151)
    z = lambda: np.zeros(rf_taps - 1)  # noqa: E731
    state_i, state_q, state_phase = z(), z(), 0
    pre_state_extract, square_state, lpf_3k_state, lpf_3k_state_Q = z(), z(), z(), z()
    anti_img_state, anti_img_state_Q, rrc_state, rrc_state_Q = z(), z(), z(), z()
    state_Pll = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    res = {}
    block_count = 0
    while (block_count + 1) * block_size < len(iq_data):
        b0, b1 = block_count * block_size, (block_count + 1) * block_size
        i_filt, state_i = signal.lfilter(rf_coeff, 1.0, iq_data[b0:b1:2], zi=state_i)
        q_filt, state_q = signal.lfilter(rf_coeff, 1.0, iq_data[b0 + 1:b1:2], zi=state_q)
        fm_demod, state_phase = fmDemodArctan(i_filt[::10], q_filt[::10], state_phase)
        extract_rds, pre_state_extract = signal.lfilter(extract_RDS_coeff, 1.0, fm_demod, zi=pre_state_extract)
        squared_rds = np.square(extract_rds)
        pre_Pll_rds, square_state = signal.lfilter(square_coeff, 1.0, squared_rds, zi=square_state)
        q0 = ncoq0(state_Pll, 114000, 240000, 0.5, phase_adj)
        post_Pll, post_Pll_Q, state_Pll = fmPll(pre_Pll_rds, 114000, 240000, state_Pll, ncoScale=0.5,
                                                phaseAdjust=phase_adj, normBandwidth=0.001)
        post_Pll_Q[0] = q0
        mixed_rds = np.multiply(extract_rds, post_Pll[0:len(extract_rds):1]) * 2
        mixed_rds_Q = np.multiply(extract_rds, post_Pll_Q[0:len(extract_rds):1]) * 2
        lpf_filt_rds, lpf_3k_state = signal.lfilter(lpf_coeff_rds, 1.0, mixed_rds, zi=lpf_3k_state)
        lpf_filt_rds_Q, lpf_3k_state_Q = signal.lfilter(lpf_coeff_rds, 1.0, mixed_rds_Q, zi=lpf_3k_state_Q)
        upsample_rds = np.zeros(len(lpf_filt_rds) * 19)
        upsample_rds_Q = np.zeros(len(lpf_filt_rds) * 19)
        for i in range(len(lpf_filt_rds)):
            upsample_rds[i * 19] = lpf_filt_rds[i]
            upsample_rds_Q[i * 19] = lpf_filt_rds_Q[i]
        anti_img, anti_img_state = signal.lfilter(anti_img_coeff, 1.0, upsample_rds, zi=anti_img_state)
        anti_img_Q, anti_img_state_Q = signal.lfilter(anti_img_coeff, 1.0, upsample_rds_Q, zi=anti_img_state_Q)
        resample_rds = anti_img[::80] * 19
        resample_rds_Q = anti_img_Q[::80] * 19
        rrc_rds, rrc_state = signal.lfilter(rrc_coeff, 1.0, resample_rds, zi=rrc_state)
        rrc_rds_Q, rrc_state_Q = signal.lfilter(rrc_coeff, 1.0, resample_rds_Q, zi=rrc_state_Q)
        r = dict(demod=fm_demod, extract=extract_rds, pre_pll=pre_Pll_rds, nco_i=post_Pll, nco_q=post_Pll_Q,
                 lpf_i=lpf_filt_rds, lpf_q=lpf_filt_rds_Q, resample_i=resample_rds, resample_q=resample_rds_Q,
                 rrc_i=rrc_rds, rrc_q=rrc_rds_Q, pll_state=np.array(state_Pll, dtype=np.float64),
                 phase=np.array([state_phase]))
        for k, v in r.items():
            res.setdefault(k, []).append(np.asarray(v, dtype=np.float64))
        block_count += 1
    assert block_count == nblocks_full
    return {k: np.stack(v) for k, v in res.items()}


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"{name}: {os.path.getsize(path) / 1e6:.2f} MB")


def main():
    # ---- config C3/C4: fmMonoBlock, block 51 200 complex, f32 IQ -----------------------
    B = 51200
    nb = 3
    iq = rtsdr.synth.fm_iq(nb * B + 1, seed=0)      # +1 sample so the strict '<' (:80) keeps nb blocks
    for taps, stereo in ((101, False), (151, True)):
        out = mono_loop(iq, 2 * B, taps, stereo)
        assert out["demod"].shape[0] == nb
        save(f"mono_t{taps}.npz", iq=iq if taps == 101 else np.zeros(0, np.float32), block=np.array([B]), **out)

    # ---- config C5 DSP: fmRDSblock, 307 200 u8 values per block --------------------------
    nbr = 2
    iq8 = rtsdr.synth.fm_iq(nbr * 153600 + 1, seed=5, dtype=np.uint8)
    out = rds_loop(iq8.astype(np.float64), 307200, nbr)
    keep = {k: v for k, v in out.items()}
    save("rds_u8.npz", iq=iq8, **keep)

    # ---- config C1: fmMonoBasic single pass (101 taps) ------------------------------------
    iqb = rtsdr.synth.fm_iq(60000, seed=3)
    rf_coeff = signal.firwin(101, 100e3 / (2.4e6 / 2), window=('hann'))
    audio_coeff = signal.firwin(151, 16e3 / (240e3 / 2), window=('hann'))
    i_filt = signal.lfilter(rf_coeff, 1.0, iqb[0::2])
    q_filt = signal.lfilter(rf_coeff, 1.0, iqb[1::2])
    fm_demod, _ = fmDemodArctan(i_filt[::10], q_filt[::10])
    audio_data = signal.lfilter(audio_coeff, 1.0, fm_demod)[::5]
    save("basic_t101.npz", iq=iqb, demod=fm_demod, audio=audio_data, wav=np.int16((audio_data / 2) * 32767))

    # ---- unit vectors: demod edge cases, lfilter edge cases, PLL, design, my_convoloution --
    rng = np.random.default_rng(11)
    cases = {}
    # demod: near-pi jumps, exact zeros, large accumulated prev phase, negative zeros
    ang = np.cumsum(rng.uniform(-3.0, 3.0, 400))
    I = np.cos(ang) * rng.uniform(0.1, 2, 400)
    Q = np.sin(ang) * rng.uniform(0.1, 2, 400)
    I[10:13] = 0.0
    Q[10:12] = 0.0
    Q[50] = -0.0
    I[60], Q[60] = -1.0, 0.0
    I[61], Q[61] = -1.0, -0.0
    for j, prev in enumerate((0.0, 1234.5678, -3.2, 3.14159)):
        d, p = fmDemodArctan(I, Q, prev)
        cases[f"demod{j}_d"] = d
        cases[f"demod{j}_prev_in"] = np.array([prev])
        cases[f"demod{j}_prev_out"] = np.array([p])
    cases["demod_I"], cases["demod_Q"] = I, Q
    # lfilter: short blocks (N < taps-1), N not a multiple of decim, random state
    for taps in (101, 151):
        b = signal.firwin(taps, 0.1, window=('hann'))
        for n in (1, 7, 99, 150, 151, 1000, 5123):
            x = rng.standard_normal(n).astype(np.float32)
            zi = rng.standard_normal(taps - 1) * 0.1
            y, zf = signal.lfilter(b, 1.0, x, zi=zi)
            cases[f"lf_t{taps}_n{n}_x"] = x
            cases[f"lf_t{taps}_n{n}_zi"] = zi
            cases[f"lf_t{taps}_n{n}_y"] = y
            cases[f"lf_t{taps}_n{n}_zf"] = zf
    # PLL alone: stereo configuration on a noisy pilot, two chained calls
    t = np.arange(6000) / 240e3
    pilot = 0.1 * np.cos(2 * np.pi * 19e3 * t + 0.3) + 0.01 * rng.standard_normal(6000)
    st = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    for j, (a, b_) in enumerate(((0, 2500), (2500, 6000))):
        q0 = ncoq0(st, 19e3, 240e3, 2.0, 0.0)
        nco, ncoq, st = fmPll(pilot[a:b_], 19e3, 240e3, st, 2)
        ncoq[0] = q0
        cases[f"pll{j}_nco"], cases[f"pll{j}_ncoq"] = nco, ncoq
        cases[f"pll{j}_state"] = np.array(st, dtype=np.float64)
    cases["pll_in"] = pilot
    # design
    cases["rrc_57000_151"] = impulseResponseRootRaisedCosine(57000, 151)
    cases["myfir_16k_240k_151"] = my_filterImpulseResponse(16e3, 240e3, 151)
    # my_convoloution: raw-history state, default 10-element history and a full one
    h = signal.firwin(31, 0.2, window=('hann'))
    x1 = rng.standard_normal(64)
    zw = rng.standard_normal(16)  # shorter than taps-1: exercises the negative-index wrap
    y1, z1 = my_convoloution(x1, h, 31, zw)
    zfull = rng.standard_normal(30)
    y2, z2 = my_convoloution(x1, h, 31, zfull)
    cases.update(myconv_zw=zw, myconv_zfull=zfull, myconv_h=h, myconv_x=x1, myconv_y1=y1, myconv_z1=z1, myconv_y2=y2, myconv_z2=z2)
    save("units.npz", **cases)

    versions = dict(python=platform.python_version(), numpy=np.__version__, scipy=scipy.__version__,
                    reference="m1nty/Real-Time-Software-Defined-Radio @ /root/reference (model/*.py)",
                    generator="tests/golden/make_golden.py")
    with open(os.path.join(HERE, "VERSIONS.json"), "w") as f:
        json.dump(versions, f, indent=2)
    print(versions)


if __name__ == "__main__":
    main()
