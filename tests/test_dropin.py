"""The drop-in claim end to end: the block loop of model/fmMonoBlock.py:80-173, statement by
statement, with only its DSP calls swapped for this package's -- `signal.lfilter` (full rate,
on the strided views iq[b0:b1:2] and iq[b0+1:b1:2], then [::10] / [::5] on the host, as the
reference slices), `fmDemodArctan` and `fmPll` -- against the golden outputs the reference's
own functions produced (tests/golden/mono_t{101,151}.npz, make_golden.py).  Coefficient
design stays scipy.signal.firwin, as in the reference.  Two documented fixes of the loop are
applied, as in the fixtures: fmPll's three return values are unpacked
(:119 unpacks two) and the combiner writes separate L/R arrays (:166-170 aliases them).
"""
import types

import numpy as np
import pytest
from scipy import signal as scipy_signal

from conftest import maxabs, rms

pytestmark = pytest.mark.gpu


def reference_loop(signal, fmDemodArctan, fmPll, iq_data, rf_taps, nblocks, stereo):
    """model/fmMonoBlock.py:22-173 with `signal`, `fmDemodArctan`, `fmPll` injected."""
    rf_Fs, rf_Fc, rf_decim = 2.4e6, 100e3, 10                              # :22-25
    audio_Fs, audio_decim, audio_taps, audio_Fc = 240e3, 5, 151, 16e3      # :28-31
    rf_coeff = signal.firwin(rf_taps, rf_Fc / (rf_Fs / 2), window=('hann'))               # :43
    audio_coeff = signal.firwin(audio_taps, audio_Fc / (audio_Fs / 2), window=('hann'))   # :45
    block_size = 1024 * rf_decim * audio_decim * 2                         # :53
    block_count = 0
    state_i_lpf_100k = np.zeros(rf_taps - 1)
    state_q_lpf_100k = np.zeros(rf_taps - 1)
    state_phase = 0
    audio_pre_state = np.zeros(audio_taps - 1)
    state_recovery = np.zeros(rf_taps - 1)
    state_extraction = np.zeros(rf_taps - 1)
    stereo_pre_state = np.zeros(audio_taps - 1)
    recovery_state = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]                       # :76
    out = []
    while (block_count + 1) * block_size < len(iq_data) and block_count < nblocks:   # :80
        r = {}
        i_filt, state_i_lpf_100k = signal.lfilter(rf_coeff, 1.0,
                                                  iq_data[(block_count) * block_size:(block_count + 1) * block_size:2],
                                                  zi=state_i_lpf_100k)
        q_filt, state_q_lpf_100k = signal.lfilter(rf_coeff, 1.0,
                                                  iq_data[(block_count) * block_size + 1:(block_count + 1) * block_size:2],
                                                  zi=state_q_lpf_100k)
        i_ds = i_filt[::rf_decim]                                          # :94-95
        q_ds = q_filt[::rf_decim]
        fm_demod, state_phase = fmDemodArctan(i_ds, q_ds, state_phase)     # :98
        audio_filt, audio_pre_state = signal.lfilter(audio_coeff, 1.0, fm_demod, zi=audio_pre_state)   # :101
        audio_block = audio_filt[::audio_decim]                            # :105
        r.update(i_ds=i_ds, q_ds=q_ds, demod=fm_demod, audio=audio_block, phase=state_phase,
                 zi_i=state_i_lpf_100k, audio_zi=audio_pre_state)
        if stereo:
            bpcoeff_recovery = signal.firwin(rf_taps, [18.5e3 / (audio_Fs / 2), 19.5e3 / (audio_Fs / 2)],
                                             window=('hann'), pass_zero="bandpass")                       # :115
            bpf_recovery, state_recovery = signal.lfilter(bpcoeff_recovery, 1.0, fm_demod, zi=state_recovery)  # :117
            recovery_pll, _, recovery_state = fmPll(bpf_recovery, 19e3, 240e3, recovery_state, 2)          # :119
            bpcoeff_extraction = signal.firwin(rf_taps, [22e3 / (audio_Fs / 2), 54e3 / (audio_Fs / 2)],
                                               window=('hann'), pass_zero="bandpass")                     # :150
            bpf_extraction, state_extraction = signal.lfilter(bpcoeff_extraction, 1.0, fm_demod,
                                                              zi=state_extraction)                        # :151
            mixed = np.multiply(recovery_pll[0:len(bpf_extraction):1], bpf_extraction)                     # :155
            mixed = mixed * 2
            stereo_coeff = signal.firwin(rf_taps, 16e3 / (audio_Fs / 2), window=('hann'))                  # :159
            stereo_filt, stereo_pre_state = signal.lfilter(stereo_coeff, 1.0, mixed, zi=stereo_pre_state)  # :160
            stereo_block = stereo_filt[::5]
            combined_l_block = (audio_block + stereo_block) / 2                                            # :166-170
            combined_r_block = (audio_block - stereo_block) / 2
            r.update(bpf_recovery=bpf_recovery, nco=recovery_pll, bpf_extraction=bpf_extraction, stereo=stereo_block,
                     left=combined_l_block, right=combined_r_block, pll_state=list(recovery_state))
        out.append(r)
        block_count += 1
    return out


@pytest.mark.parametrize("taps", [101, 151])
def test_fmMonoBlock_loop_through_the_shim(sdr, gpu_ctx, golden, taps):
    g = golden(f"mono_t{taps}.npz")
    iq = golden("mono_t101.npz")["iq"]                   # both fixtures were made from this IQ
    shim = types.SimpleNamespace(lfilter=sdr.lfilter, firwin=scipy_signal.firwin)
    stereo = taps == 151
    got = reference_loop(shim, sdr.fmDemodArctan, sdr.fmPll, iq, taps, 3, stereo)
    assert len(got) == 3
    for k, r in enumerate(got):
        # decimation indices: output m of [::10] is input 10 m (exact lengths and values)
        assert r["i_ds"].shape == g["i_ds"][k].shape and maxabs(r["i_ds"], g["i_ds"][k]) < 2e-6
        assert maxabs(r["q_ds"], g["q_ds"][k]) < 2e-6
        assert rms(r["demod"], g["demod"][k]) < 1e-6 and maxabs(r["demod"], g["demod"][k]) < 1e-5
        assert r["audio"].shape == g["audio"][k].shape
        assert rms(r["audio"], g["audio"][k]) < 1e-6 and maxabs(r["audio"], g["audio"][k]) < 1e-5
        assert abs(r["phase"] - g["phase"][k][0]) < 1e-5
        assert maxabs(r["zi_i"], g["zi_i"][k]) < 1e-12         # lfilter state from exact f32 IQ, in f64
        assert maxabs(r["audio_zi"], g["audio_zi"][k]) < 1e-6
        if stereo:
            assert maxabs(r["nco"], g["nco"][k]) < 1e-7
            assert maxabs(r["pll_state"], g["pll_state"][k]) < 1e-6
            for key in ("stereo", "left", "right"):
                assert rms(r[key], g[key][k]) < 1e-6 and maxabs(r[key], g[key][k]) < 1e-5, key
