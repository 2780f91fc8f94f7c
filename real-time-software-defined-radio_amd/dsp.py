"""Reference-named per-block functions, computed by the HIP kernels of libsdr.so.

Drop-in counterparts of the calls model/fmMonoBlock.py and model/fmRDSblock.py make
per block.  Same names, argument meaning, return shapes and error behaviour:

    lfilter(b, a, x, zi=None)                  scipy.signal.lfilter FIR branch
    fmDemodArctan(I, Q, prev_phase=0.0)        model/fmSupportLib.py:15-44
    fmPll(pllIn, freq, Fs, recovery_state, ncoScale=1.0, phaseAdjust=0.0,
          normBandwidth=0.01)                  model/fmPll.py:4-46
    my_convoloution(x, h, N_taps, my_zi)       model/fmSupportLib.py:157-176
    estimatePSD(samples, NFFT, Fs)             model/fmSupportLib.py:66-140 (Bartlett PSD)
    DFT(x)                                     model/fmSupportLib.py:46-60

plus the fused forms the hot path is built from:

    lfilter_decim(b, x, zi, decim)             lfilter(...)[::decim] in one kernel
    rf_frontend_block(iq, rf_coeff, zi_i, zi_q, prev_phase, rf_decim=10)
    mono_block(iq, rf_coeff, audio_coeff, state)
    resample(x, b, zi, up, down)               model/fmRDSblock.py:184-199
    fm_mono_streams(iq, rf_coeff, audio_coeff) model/fmMonoBasic.py:70-111 over one or
                                               more whole streams, demod kept on chip

Arrays come back as float64 (the reference's dtype) so downstream np.concatenate /
wavfile code is unchanged; the kernels compute in f32 (state in f64), see DESIGN.md.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from ._lib import SDR_IQ_F32, SDR_IQ_U8, SDR_PRE_MIX, SDR_PRE_NONE, SDR_PRE_SQUARE, c_f32, c_f64, check, f32p, f64p


def _ctx(ctx=None):
    return ctx if ctx is not None else _lib.get_context()


def _taps(b, a=1.0, max_taps=256):
    b = np.atleast_1d(np.asarray(b))
    a = np.atleast_1d(np.asarray(a))
    if b.ndim != 1 or a.ndim != 1:
        raise ValueError("object of too small depth for desired array")
    if len(a) != 1:
        raise NotImplementedError("only FIR filters (a = [a0]) are implemented on the GPU path")
    if np.iscomplexobj(b) or np.iscomplexobj(a):
        raise NotImplementedError(f"input type '{np.result_type(b, a)}' not supported")
    b = np.array(b, dtype=np.float64) / float(a[0])
    if not 1 <= len(b) <= max_taps:
        raise ValueError(f"{len(b)} taps: this GPU path supports 1..{max_taps} taps")
    return np.ascontiguousarray(b)


def _check_x(x):
    x = np.asarray(x)
    if x.ndim != 1:
        raise ValueError("only 1-D signals are supported")
    if np.iscomplexobj(x):
        raise NotImplementedError(f"input type '{x.dtype}' not supported")
    if x.dtype == object:
        raise ValueError("object arrays are not supported")
    return x


def _check_zi(zi, ntaps):
    if zi is None:
        return None
    zi = np.asarray(zi)
    if zi.ndim != 1:
        raise ValueError("object of too small depth for desired array")
    if zi.shape != (ntaps - 1,):
        raise ValueError(f"Unexpected shape for zi: expected ({ntaps - 1},), found {zi.shape}.")
    return np.array(zi, dtype=np.float64)


# ---------------------------------------------------------------------------------
def lfilter_decim(b, x, zi=None, decim: int = 1, *, pre: int = SDR_PRE_NONE, mix=None,
                  gain: float = 1.0, ctx=None):
    """lfilter(b, 1.0, pre(x), zi)[::decim] computed only at the kept outputs.

    Returns (y, zf) when zi is given, else y (scipy's convention)."""
    b = _taps(b)
    x = c_f32(_check_x(x))
    zi = _check_zi(zi, len(b))
    c = _ctx(ctx)
    n = x.shape[0]
    y = np.empty((n + decim - 1) // decim, dtype=np.float32)
    zf = zi.copy() if zi is not None else None
    mx = None
    if pre == SDR_PRE_MIX:
        mx = c_f32(mix)
        if mx.shape[0] < n:
            raise ValueError("mix operand shorter than x")
    check(c.lib.sdr_lfilter(c.handle, f32p(x), f32p(mx), float(gain), int(pre), n, f64p(b), len(b),
                            int(decim), f64p(zf), f32p(y)), "sdr_lfilter")
    y = y.astype(np.float64)
    return (y, zf) if zi is not None else y


def lfilter(b, a, x, zi=None, ctx=None):
    """scipy.signal.lfilter for FIR b (a scalar), as called at model/fmMonoBlock.py:86-91."""
    b = _taps(b, a)
    return lfilter_decim(b, x, zi, 1, ctx=ctx)


def fmDemodArctan(I, Q, prev_phase=0.0, ctx=None):
    """(fm_demod, prev_phase) of model/fmSupportLib.py:15-44 (atan2 + np.unwrap step)."""
    I = c_f32(_check_x(I))
    Q = c_f32(_check_x(Q))
    if I.shape != Q.shape:
        raise ValueError("I and Q must have the same length")
    c = _ctx(ctx)
    out = np.empty(I.shape[0], dtype=np.float32)
    ph = np.array([float(prev_phase)], dtype=np.float64)
    check(c.lib.sdr_fm_demod(c.handle, f32p(I), f32p(Q), I.shape[0], f64p(ph), f32p(out)), "sdr_fm_demod")
    return out.astype(np.float64), float(ph[0])


def fmPll(pllIn, freq, Fs, recovery_state, ncoScale=1.0, phaseAdjust=0.0, normBandwidth=0.01, ctx=None):
    """(ncoOut, ncoOutQ, recovery_state) of model/fmPll.py:4-46.

    recovery_state = [integrator, phaseEst, feedbackI, feedbackQ, ncoOut[0], trigOffset]
    is updated in place (as the reference does) and returned.  ncoOutQ[0], left
    uninitialised by the reference (np.empty), is the carried quadrature value."""
    x = c_f32(_check_x(pllIn))
    if len(recovery_state) != 6:
        raise ValueError("recovery_state must have 6 elements")
    st = np.array([float(v) for v in recovery_state], dtype=np.float64)
    c = _ctx(ctx)
    n = x.shape[0]
    nco = np.empty(n + 1, dtype=np.float32)
    ncoq = np.empty(n + 1, dtype=np.float32)
    check(c.lib.sdr_pll(c.handle, f32p(x), n, float(freq), float(Fs), float(ncoScale), float(phaseAdjust),
                        float(normBandwidth), f64p(st), f32p(nco), f32p(ncoq)), "sdr_pll")
    for i in range(6):
        recovery_state[i] = float(st[i])
    return nco.astype(np.float64), ncoq.astype(np.float64), recovery_state


def history_from_my_zi(my_zi, T):
    """Raw pre-history h[j] = x[j-(T-1)], j = 0..T-2, as model/fmSupportLib.py:164-172
    reads it: x[n-k] (n-k < 0) comes from my_zi[len(my_zi)-1-count] with
    count = k-n-1, i.e. my_zi[len + (n-k)] -- Python's negative-index wrap included,
    IndexError where the reference would raise one."""
    zi = np.asarray(my_zi, dtype=np.float64)
    L = len(zi)
    hist = np.zeros(max(T - 1, 0), dtype=np.float64)
    for j in range(T - 1):
        idx = L + (j - (T - 1))
        if -L <= idx < L:
            hist[j] = zi[idx]
        elif L:
            raise IndexError(f"index {idx} is out of bounds for axis 0 with size {L}")
    return hist


def my_convoloution(x, h, N_taps, my_zi=None, ctx=None):
    """(y, zi) of model/fmSupportLib.py:157-176: FIR whose state is the raw input history.

    Out-of-block samples x[n-k] (n-k < 0) are read from my_zi[len(my_zi)-1-count]
    exactly as the reference indexes them (including Python's negative-index wrap
    for a history shorter than the filter), then the GPU FIR runs over
    [history, x]; the new state is x[-len(my_zi):]."""
    h = _taps(h)  # the reference loops over len(h); N_taps is unused there too
    x = _check_x(x)
    zi = np.zeros(10) if my_zi is None else np.asarray(my_zi, dtype=np.float64)
    T = len(h)
    L = len(zi)
    n = len(x)
    xd = np.asarray(x, dtype=np.float64)
    # the new state is x[-len(my_zi):] (:175); for an empty my_zi that is x[-0:], the whole block
    new_zi = xd[-L:] if L else xd[0:]
    if n == 0:                       # no output sample reads the history
        return np.zeros(0), new_zi
    if L == 0 and T > 1:             # y[0] reads my_zi[len(my_zi)-1-0] = my_zi[-1] (:169)
        raise IndexError("index -1 is out of bounds for axis 0 with size 0")
    hist = history_from_my_zi(zi, T)
    full = np.concatenate([hist, xd]).astype(np.float32)
    c = _ctx(ctx)
    buf = _lib.DeviceBuffer.from_array(c, full)
    out = _lib.DeviceBuffer(c, max(4 * n, 16))
    check(c.lib.sdr_fir_dev(c.handle, buf.ptr + 4 * (T - 1), None, 1.0, SDR_PRE_NONE, n, n, T - 1, 1,
                            f64p(h), T, 1, None, 0, None, out.ptr, n), "sdr_fir_dev")
    y = out.download(n).astype(np.float64)
    return y, new_zi


def resample(x, b, zi=None, up: int = 19, down: int = 80, ctx=None):
    """lfilter(b, 1, zero_stuff(x, up), zi)[::down] * up (model/fmRDSblock.py:184-199; the
    mode-1 24/125 audio resampler, src/filter.cpp:222-298, is y / up).  Up to 4096 taps."""
    b = _taps(b, max_taps=4096)
    x = c_f32(_check_x(x))
    zi = _check_zi(zi, len(b))
    c = _ctx(ctx)
    n = x.shape[0]
    y = np.empty((n * up + down - 1) // down, dtype=np.float32)
    zf = zi.copy() if zi is not None else None
    check(c.lib.sdr_resample(c.handle, f32p(x), n, f64p(b), len(b), int(up), int(down), f64p(zf), f32p(y)),
          "sdr_resample")
    y = y.astype(np.float64)
    return (y, zf) if zi is not None else y


def _iq_args(iq):
    iq = np.asarray(iq)
    if iq.ndim != 1 or iq.shape[0] % 2:
        raise ValueError("iq must be a 1-D interleaved [I0, Q0, I1, Q1, ...] array")
    if iq.dtype == np.uint8:
        return np.ascontiguousarray(iq), SDR_IQ_U8
    return c_f32(iq), SDR_IQ_F32


def rf_frontend_block(iq, rf_coeff, zi_i=None, zi_q=None, prev_phase=0.0, rf_decim=10,
                      return_iq=False, ctx=None):
    """One block of model/fmMonoBlock.py:86-98 in a single fused kernel.

    iq: interleaved float32 (model/fmMonoBlock.py:39) or uint8 (model/fmRDSblock.py:58,
    normalised (x-128)/128 on the GPU).  Returns (fm_demod, zi_i, zi_q, prev_phase)
    [+ (i_ds, q_ds) if return_iq]."""
    b = _taps(rf_coeff)
    iq, dt = _iq_args(iq)
    n = iq.shape[0] // 2
    zi_i = _check_zi(np.zeros(len(b) - 1) if zi_i is None else zi_i, len(b))
    zi_q = _check_zi(np.zeros(len(b) - 1) if zi_q is None else zi_q, len(b))
    c = _ctx(ctx)
    m = (n + rf_decim - 1) // rf_decim
    demod = np.empty(m, dtype=np.float32)
    i_ds = np.empty(m, dtype=np.float32) if return_iq else None
    q_ds = np.empty(m, dtype=np.float32) if return_iq else None
    ph = np.array([float(prev_phase)])
    check(c.lib.sdr_rf_frontend(c.handle, iq.ctypes.data, dt, n, f64p(b), len(b), int(rf_decim), f64p(zi_i),
                                f64p(zi_q), f64p(ph), f32p(demod), f32p(i_ds), f32p(q_ds)), "sdr_rf_frontend")
    out = (demod.astype(np.float64), zi_i, zi_q, float(ph[0]))
    if return_iq:
        out = out + (i_ds.astype(np.float64), q_ds.astype(np.float64))
    return out


class MonoState:
    """Per-stream carry of model/fmMonoBlock.py:57-67: RF zi (I, Q), demod phase, audio zi."""

    def __init__(self, rf_taps=151, audio_taps=151):
        self.zi_i = np.zeros(rf_taps - 1)
        self.zi_q = np.zeros(rf_taps - 1)
        self.phase = 0.0
        self.audio_zi = np.zeros(audio_taps - 1)


def mono_block(iq, rf_coeff, audio_coeff, state: MonoState, rf_decim=10, audio_decim=5,
               return_demod=False, ctx=None):
    """One iteration of model/fmMonoBlock.py:86-105 (FE + audio LPF + [::5]) on the GPU.

    The demod stream stays in HBM between the two kernels.  Updates `state` in place
    and returns audio_block (float64) [+ fm_demod]."""
    b = _taps(rf_coeff)
    ab = _taps(audio_coeff)
    iq, dt = _iq_args(iq)
    n = iq.shape[0] // 2
    for name, ln in (("zi_i", len(b)), ("zi_q", len(b)), ("audio_zi", len(ab))):
        setattr(state, name, _check_zi(getattr(state, name), ln))
    c = _ctx(ctx)
    m = (n + rf_decim - 1) // rf_decim
    a = (m + audio_decim - 1) // audio_decim
    audio = np.empty(a, dtype=np.float32)
    demod = np.empty(m, dtype=np.float32) if return_demod else None
    ph = np.array([float(state.phase)])
    check(c.lib.sdr_mono_block(c.handle, iq.ctypes.data, dt, n, f64p(b), len(b), int(rf_decim),
                               f64p(state.zi_i), f64p(state.zi_q), f64p(ph), f64p(ab), len(ab),
                               int(audio_decim), f64p(state.audio_zi), f32p(demod), f32p(audio)),
          "sdr_mono_block")
    state.phase = float(ph[0])
    audio = audio.astype(np.float64)
    return (audio, demod.astype(np.float64)) if return_demod else audio


def fm_mono_streams(iq, rf_coeff, audio_coeff, rf_decim=10, audio_decim=5, ctx=None):
    """Whole-capture mono receiver of model/fmMonoBasic.py:70-111 (lfilter without state,
    [::rf_decim], fmDemodArctan from phase 0, audio lfilter, [::audio_decim]) for each row
    of `iq` (1-D: one stream; 2-D: streams x interleaved samples), in one fused kernel
    (sdr_fe_mono_dev): the demodulated signal never leaves the CU.  Returns float64 audio
    of shape (ceil(ceil(n / rf_decim) / audio_decim),) or (streams, that)."""
    b = _taps(rf_coeff)
    ab = _taps(audio_coeff)
    iq = np.asarray(iq)
    one = iq.ndim == 1
    iq2 = iq[None, :] if one else iq
    if iq2.ndim != 2 or iq2.shape[1] % 2:
        raise ValueError("iq must be [I0, Q0, ...] rows of even length")
    rows = [_iq_args(r) for r in iq2]
    dt = rows[0][1]
    data = np.ascontiguousarray(np.stack([r[0] for r in rows])) if rows else iq2
    S, n = data.shape[0], data.shape[1] // 2
    c = _ctx(ctx)
    m = (n + rf_decim - 1) // rf_decim
    a = (m + audio_decim - 1) // audio_decim
    astride = a + (a & 1)
    d_iq = _lib.DeviceBuffer.from_array(c, data)
    d_au = _lib.DeviceBuffer(c, 4 * max(astride * S, 4))
    try:
        check(c.lib.sdr_fe_mono_dev(c.handle, d_iq.ptr, dt, n, n, S, f64p(b), len(b), int(rf_decim), f64p(ab),
                                    len(ab), int(audio_decim), d_au.ptr, astride), "sdr_fe_mono_dev")
        out = d_au.download(astride * S).reshape(S, astride)[:, :a].astype(np.float64)
    finally:
        d_iq.free()
        d_au.free()
    return out[0] if one else out


def split_halo(rf_taps: int, audio_taps: int, rf_decim: int = 10, audio_decim: int = 5) -> int:
    """IQ samples a range of one stream reads before its start when the stream is split
    (SURVEY §8e): audio sample j depends on IQ [D*A*j - ((rf_taps-1) + rf_decim*audio_taps),
    D*A*j], so (rf_taps-1) + rf_decim*audio_taps, rounded up to a whole audio sample
    (rf_decim*audio_decim IQ samples)."""
    step = rf_decim * audio_decim
    need = (rf_taps - 1) + rf_decim * audio_taps
    return (need + step - 1) // step * step


def fm_mono_range(iq, start, end, rf_coeff, audio_coeff, rf_decim=10, audio_decim=5, ctx=None):
    """The audio of IQ samples [start, end) of one stream, identical to those samples'
    outputs of fm_mono_streams(iq) (the whole-stream pass), computed from the range plus a
    read-only halo of split_halo(...) samples before it: one range per GPU, no exchange
    (SURVEY §8e).  start must be a multiple of rf_decim*audio_decim; the outputs are those
    audio samples j whose IQ position rf_decim*audio_decim*j lies in [start, end)."""
    step = rf_decim * audio_decim
    iq = np.asarray(iq)
    n = iq.shape[0] // 2
    if start % step or not (0 <= start <= end <= n):
        raise ValueError(f"range [{start}, {end}) of {n}: start must be a multiple of {step}")
    h = split_halo(len(_taps(rf_coeff)), len(_taps(audio_coeff)), rf_decim, audio_decim)
    w0 = max(0, start - h)
    a = fm_mono_streams(iq[2 * w0:2 * end], rf_coeff, audio_coeff, rf_decim, audio_decim, ctx=ctx)
    j0 = (start - w0) // step
    j1 = (end - w0 + step - 1) // step
    return a[j0:j1]


def estimatePSD(samples, NFFT, Fs, ctx=None):
    """(freq, psd_est) of model/fmSupportLib.py:66-140: Bartlett estimate over
    floor(len/NFFT) non-overlapping Hann-windowed segments, per-segment dB averaged.
    The segments' FFTs and dB values run in f64 on the GPU (sdr_psd); NFFT must be a power
    of two <= 4096.  A zero-power bin raises ValueError like the reference's math.log10."""
    x = _check_x(samples).astype(np.float64)
    nfft = int(NFFT)
    freq = np.arange(0, Fs / 2, Fs / nfft)
    psd = np.empty(nfft // 2, dtype=np.float64)
    c = _ctx(ctx)
    check(c.lib.sdr_psd(c.handle, f64p(c_f64(x)), x.shape[0], nfft, float(Fs), f64p(psd)), "sdr_psd")
    return freq, psd


def DFT(x, ctx=None):
    """Xf of model/fmSupportLib.py:46-60 (direct O(N^2) DFT, complex128), on the GPU."""
    x = c_f64(_check_x(x).astype(np.float64))
    out = np.empty(2 * x.shape[0], dtype=np.float64)
    c = _ctx(ctx)
    check(c.lib.sdr_dft(c.handle, f64p(x), x.shape[0], f64p(out)), "sdr_dft")
    return out.view(np.complex128)
