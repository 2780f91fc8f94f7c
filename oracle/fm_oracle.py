"""ORACLE — test infrastructure only (never imported by the product package).

CPU restatement, in float64 numpy, of the reference's per-block signal path, used
as the checker for the HIP kernels.  Only tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg may import this module.

Pinning: the restatement is checked against golden vectors produced by running
the reference's own functions (model/fmSupportLib.fmDemodArctan, model/fmPll.fmPll,
model/fmRRC.impulseResponseRootRaisedCosine) and scipy.signal.lfilter/firwin in the
reference's block loops -- tests/golden/make_golden.py, fixtures in tests/golden/.
The reference ships no test vectors of its own, so these fixtures are
the pin.

Each function cites the reference lines it restates.
"""
from __future__ import annotations

import math

import numpy as np
from scipy import signal


# ---- filtering ----------------------------------------------------------------------
def lfilter_fir(b, x, zi=None):
    """scipy.signal.lfilter(b, 1.0, x, zi) FIR branch, scipy 1.15.3
    _signaltools.py:2153-2172: full = convolve(b, x); full[:T-1] += zi; y = full[:N];
    zf = full[N:].  As called at model/fmMonoBlock.py:86-91,101,117,151,160."""
    b = np.asarray(b, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    full = np.convolve(b, x)
    if zi is not None:
        zi = np.asarray(zi, dtype=np.float64)
        full[:len(zi)] += zi
    n = len(x)
    y = full[:n]
    return (y, full[n:].copy()) if zi is not None else y


def lfilter_decim(b, x, zi, decim):
    """lfilter(...)[::decim] (model/fmMonoBlock.py:94-95,105) and the final state, computing
    only the kept outputs (the checker's speed: scipy.signal.upfirdn, the same sums as
    lfilter_fir's in another order -- tests/test_oracle.py::test_decim_and_resample_fast_forms)."""
    b = np.asarray(b, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    T, n = len(b), len(x)
    y = signal.upfirdn(b, x, 1, decim)[:(n + decim - 1) // decim] if n else np.zeros(0)
    zi = np.zeros(T - 1) if zi is None else np.asarray(zi, dtype=np.float64)
    m = np.arange(0, min(n, T - 1), decim)
    y[m // decim] += zi[m]
    k = np.arange(T - 1)
    zf = np.where(n + k < T - 1, zi[np.minimum(n + k, T - 2)], 0.0)
    idx = n - (T - 1) + k                                  # the last T - 1 inputs (zero before the start)
    tail = np.where(idx >= 0, x[np.clip(idx, 0, max(n - 1, 0))] if n else 0.0, 0.0)
    zf = zf + np.convolve(b, tail)[T - 1:2 * T - 2]
    return y, zf


def resample_literal(x, b, zi, up, down):
    """Zero-stuff by `up`, anti-image lfilter, [::down] * up (model/fmRDSblock.py:184-199),
    literally (the zero-stuffed stream through lfilter_fir)."""
    u = np.zeros(len(x) * up)
    u[::up] = x
    y, zf = lfilter_fir(b, u, zi)
    return y[::down] * up, zf


def resample(x, b, zi, up, down):
    """resample_literal's values computed polyphase (the checker's speed: only the taps that meet
    a nonzero stuffed sample are summed, up times fewer products; the same sums in another
    order -- tests/test_oracle.py::test_resample_polyphase_equals_literal): output n of the
    stuffed stream is sum_i b[n mod up + up i] x[n // up - i] (+ zi[n], n < T - 1), its final
    state zf[k] = sum_{j > k, j = N + k mod up} b[j] x[(N + k - j) / up] (+ zi[N + k])."""
    b = np.asarray(b, dtype=np.float64)
    x = np.asarray(x, dtype=np.float64)
    T, nx = len(b), len(x)
    N = nx * up
    n = np.arange(0, N, down)
    r, q = n % up, n // up
    y = np.zeros(len(n))
    for i in range((T + up - 1) // up):
        j = r + up * i
        qi = q - i
        ok = (j < T) & (qi >= 0)
        y[ok] += b[j[ok]] * x[qi[ok]]
    zi = np.asarray(zi, dtype=np.float64)
    head = n < T - 1
    y[head] += zi[n[head]]
    k = np.arange(T - 1)
    zf = np.where(N + k < T - 1, zi[np.minimum(N + k, T - 2)], 0.0)
    # the stuffed stream's last T - 1 samples (zero before its start): zf = (b * tail)[T-1 .. 2T-3]
    m = N - (T - 1) + k
    tail = np.where((m >= 0) & (m % up == 0), x[np.clip(m // up, 0, nx - 1)] if nx else 0.0, 0.0)
    zf = zf + np.convolve(b, tail)[T - 1:2 * T - 2]
    return y * up, zf


# ---- FM discriminator ---------------------------------------------------------------
def fm_demod_arctan_loop(I, Q, prev_phase=0.0):
    """Literal per-sample restatement of model/fmSupportLib.py:15-44 (small inputs)."""
    out = np.empty(len(I))
    for k in range(len(I)):
        cur = math.atan2(Q[k], I[k])
        prev_phase, cur = np.unwrap([prev_phase, cur])
        out[k] = cur - prev_phase
        prev_phase = cur
    return out, prev_phase


def fm_demod_arctan(I, Q, prev_phase=0.0):
    """Vectorised model/fmSupportLib.py:15-44: d_k = wrap(phi_k - phi_{k-1}) with
    np.unwrap's rule (numpy _function_base_impl.py:1790-1800); the returned state is
    the accumulated unwrapped phase prev + sum(d)."""
    phi = np.arctan2(np.asarray(Q, dtype=np.float64), np.asarray(I, dtype=np.float64))
    if len(phi) == 0:
        return np.empty(0), prev_phase
    dd = np.diff(np.concatenate([[float(prev_phase)], phi]))
    ddmod = np.mod(dd + np.pi, 2 * np.pi) - np.pi
    ddmod[(ddmod == -np.pi) & (dd > 0)] = np.pi
    d = np.where(np.abs(dd) < np.pi, dd, ddmod)
    return d, float(prev_phase) + float(np.sum(d))


# ---- PLL ------------------------------------------------------------------------------
def fm_pll(pllIn, freq, Fs, state, ncoScale=1.0, phaseAdjust=0.0, normBandwidth=0.01):
    """Restatement of model/fmPll.py:4-46 (f64, per-sample loop).  Returns
    (ncoOut, ncoOutQ, new_state); ncoOutQ[0], never written by the reference
    (np.empty at :13), is defined as sin(theta_prev*scale + adj) with theta_prev
    rebuilt from the carried state (0.0 at stream start) -- DESIGN.md §6."""
    Kp = normBandwidth * 2.666
    Ki = normBandwidth * normBandwidth * 3.555
    n = len(pllIn)
    nco = np.empty(n + 1)
    ncoq = np.empty(n + 1)
    integ, phase, fI, fQ, nco[0], off = [float(v) for v in state]
    w = 2 * math.pi * (freq / Fs)
    ncoq[0] = math.sin((w * off + phase) * ncoScale + phaseAdjust) if off > 0 else 0.0
    for k in range(n):
        e = math.atan2(pllIn[k] * (-fQ), pllIn[k] * (+fI))
        integ = integ + Ki * e
        phase = phase + Kp * e + integ
        arg = w * (off + k + 1) + phase
        fI = math.cos(arg)
        fQ = math.sin(arg)
        nco[k + 1] = math.cos(arg * ncoScale + phaseAdjust)
        ncoq[k + 1] = math.sin(arg * ncoScale + phaseAdjust)
    return nco, ncoq, [integ, phase, fI, fQ, nco[-1], off + n]


_LIBORACLE = None


def fm_pll_c(pllIn, freq, Fs, state, ncoScale=1.0, phaseAdjust=0.0, normBandwidth=0.01):
    """fm_pll through oracle/fm_oracle.c::orc_pll (the same restatement of model/fmPll.py:4-46,
    operation for operation; bit-identical to fm_pll: tests/test_oracle.py::test_c_oracle_pll).
    ~100x faster than the Python loop, for checks over hundreds of blocks.  Needs
    oracle/_build/liboracle.so (make -C oracle)."""
    global _LIBORACLE
    if _LIBORACLE is None:
        import ctypes
        import os
        lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "_build", "liboracle.so"))
        P = np.ctypeslib.ndpointer
        d = ctypes.c_double
        lib.orc_pll.argtypes = [P(np.float64), ctypes.c_int64, d, d, d, d, d, P(np.float64), P(np.float64),
                                P(np.float64)]
        lib.orc_pll.restype = None
        _LIBORACLE = lib
    x = np.ascontiguousarray(pllIn, dtype=np.float64)
    n = len(x)
    nco = np.empty(n + 1)
    ncoq = np.empty(n + 1)
    st = np.array([float(v) for v in state], dtype=np.float64)
    _LIBORACLE.orc_pll(x, n, float(freq), float(Fs), float(ncoScale), float(phaseAdjust), float(normBandwidth), st,
                       nco, ncoq)
    return nco, ncoq, [float(v) for v in st]


# ---- tap design (model/fmRRC.py:12-47) --------------------------------------------------
def rrc_taps(Fs, N_taps):
    Ts, beta = 1 / 2375.0, 0.90
    h = np.empty(N_taps)
    for k in range(N_taps):
        t = float(k - N_taps / 2) / Fs
        if t == 0.0:
            h[k] = 1.0 + beta * (4 / math.pi - 1)
        elif t == -Ts / (4 * beta) or t == Ts / (4 * beta):
            q = math.pi / (4 * beta)
            h[k] = beta / np.sqrt(2) * ((1 + 2 / math.pi) * math.sin(q) + (1 - 2 / math.pi) * math.cos(q))
        else:
            x = 4 * beta * t / Ts
            h[k] = (math.sin(math.pi * t * (1 - beta) / Ts) + x * math.cos(math.pi * t * (1 + beta) / Ts)) / \
                   (math.pi * t * (1 - x * x) / Ts)
    return h


# ---- block loops --------------------------------------------------------------------------
def mono_coeffs(rf_taps=151, audio_taps=151):
    """model/fmMonoBlock.py:43-45."""
    return (signal.firwin(rf_taps, 100e3 / (2.4e6 / 2), window=("hann")),
            signal.firwin(audio_taps, 16e3 / (240e3 / 2), window=("hann")))


def stereo_coeffs(taps=151):
    """model/fmMonoBlock.py:115,150,159."""
    fs2 = 240e3 / 2
    return (signal.firwin(taps, [18.5e3 / fs2, 19.5e3 / fs2], window=("hann"), pass_zero="bandpass"),
            signal.firwin(taps, [22e3 / fs2, 54e3 / fs2], window=("hann"), pass_zero="bandpass"),
            signal.firwin(taps, 16e3 / fs2, window=("hann")))


def rds_coeffs(taps=151):
    """model/fmRDSblock.py:88-111."""
    fs2 = 240000 / 2
    return dict(
        extract=signal.firwin(taps, [54000 / fs2, 60000 / fs2], window=("hann"), pass_zero="bandpass"),
        square=signal.firwin(taps, [113500 / fs2, 114500 / fs2], window=("hann"), pass_zero="bandpass"),
        lpf=signal.firwin(taps, 3000 / fs2, window=("hann")),
        anti_img=signal.firwin(taps, (57000 / 2) / ((240000 * 19) / 2), window=("hann")),
        rrc=rrc_taps(57000, 151),
    )


def mono_stereo_blocks(iq, block_complex, rf_taps=151, audio_taps=151, stereo=True, nblocks=None,
                       demod_fn=fm_demod_arctan, pll_fn=fm_pll, alt_in=None, alt_from=0):
    """Restatement of the model/fmMonoBlock.py:80-173 loop (fmPll unpack fixed, intended
    combiner).  iq: interleaved float32.  Returns a list of per-block dicts.

    alt_in (test infrastructure for the device's own PLL inputs): a function k -> block k's
    pilot-BPF row to run a SECOND fmPll on (state carried from the stream start like the first)
    and the same mixer / LPF / combiner statements after it, with their own filter states; block
    k's dict then holds r["alt"] = {"nco", "stereo", "left", "right"}.  The PLL and everything
    after it depend on the PLL input only, so this chain is the reference's on that input.  Its
    downstream statements run from block alt_from - 1 on (zero filter state there: an FIR's zf
    depends only on its last taps - 1 inputs, so blocks >= alt_from are exact); the second PLL
    runs on every block (its state)."""
    rf_b, au_b = mono_coeffs(rf_taps, audio_taps)
    pil_b, ext_b, st_b = stereo_coeffs(151)
    B = 2 * block_complex
    zi_i = np.zeros(rf_taps - 1)
    zi_q = np.zeros(rf_taps - 1)
    phase = 0.0
    au_zi = np.zeros(audio_taps - 1)
    rec_zi, ext_zi = np.zeros(150), np.zeros(150)
    pll_state = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    chains = [{"pll": pll_state, "st_zi": np.zeros(150)}]
    if alt_in is not None:
        chains.append({"pll": list(pll_state), "st_zi": np.zeros(150)})

    def stereo_tail(r, c, x):
        nco, _, c["pll"] = pll_fn(x, 19e3, 240e3, list(c["pll"]), 2)
        o = {"nco": nco}
        if c is chains[0] or k >= alt_from - 1:
            mixed = np.multiply(nco[0:len(r["bpf_extraction"])], r["bpf_extraction"]) * 2
            o["stereo"], c["st_zi"] = lfilter_decim(st_b, mixed, c["st_zi"], 5)
            o["left"] = (r["audio"] + o["stereo"]) / 2
            o["right"] = (r["audio"] - o["stereo"]) / 2
        return o
    out = []
    k = 0
    while (k + 1) * B < len(iq) and (nblocks is None or k < nblocks):   # strict "<" as :80
        blk = iq[k * B:(k + 1) * B]
        r = {}
        r["i_ds"], zi_i = lfilter_decim(rf_b, blk[0::2], zi_i, 10)
        r["q_ds"], zi_q = lfilter_decim(rf_b, blk[1::2], zi_q, 10)
        r["demod"], phase = demod_fn(r["i_ds"], r["q_ds"], phase)
        r["audio"], au_zi = lfilter_decim(au_b, r["demod"], au_zi, 5)
        r["phase"] = phase
        if stereo:
            r["bpf_recovery"], rec_zi = lfilter_fir(pil_b, r["demod"], rec_zi)
            r["bpf_extraction"], ext_zi = lfilter_fir(ext_b, r["demod"], ext_zi)
            r.update(stereo_tail(r, chains[0], r["bpf_recovery"]))
            if alt_in is not None:
                r["alt"] = stereo_tail(r, chains[1], np.asarray(alt_in(k), dtype=np.float64))
        out.append(r)
        k += 1
    return out


def mode1_coeffs(rf_taps=151):
    """Mode 1 (src/fm_radio.cpp:16-21, :150-252: 2.5 MS/s RF, IF 250 kS/s, 24/125 to 48 kS/s).
    The RF low-pass and the resampler filter are the reference's (cutoff 100 kHz at 2.5 MHz;
    16 kHz at the 6 MHz upsampled rate, 3 623 taps).  The pilot and stereo band-passes are
    designed at the 250 kS/s IF they run at -- the INTENDED form: src/fm_radio.cpp:231-240
    designs them against 6 MHz, which puts both pass-bands far below 19 kHz / 22-54 kHz
    (parity unpinned)."""
    fs2 = 250e3 / 2
    return dict(rf=signal.firwin(rf_taps, 100e3 / 1.25e6, window=("hann")),
                res=signal.firwin(3623, 16e3 / 3e6, window=("hann")),
                pilot=signal.firwin(151, [18.5e3 / fs2, 19.5e3 / fs2], window=("hann"), pass_zero="bandpass"),
                ext=signal.firwin(151, [22e3 / fs2, 54e3 / fs2], window=("hann"), pass_zero="bandpass"))


def mode1_stereo_blocks(iq, block_complex=153_600, rf_taps=151, nblocks=None):
    """Mode-1 stereo in its intended form (parity UNPINNED: the reference's own mode-1 stereo,
    src/fm_radio.cpp:231-252, is defective -- band-passes designed at 6 MHz, fmPLL at Fs
    240 kHz on a 250 kS/s IF, mixer without the x2 of model/fmMonoBlock.py:154, stereo
    low-pass decimating by 5 with no upsampling, so its stereo channel has the wrong rate and
    length).  Restated here as the mode-0 stereo path (model/fmMonoBlock.py:113-166) moved to
    the 250 kS/s IF: pilot BPF -> fmPll(19 kHz, Fs 250 kHz, x2) -> stereo BPF -> mixer x2 ->
    the mode-1 mono resampler (24/125, 3 623 taps, :226-229) -> L/R = (m +- s)/2.  The FE is
    the reference's mode-1 RF stage (151 taps at 2.5 MHz, decim 10, src/fm_radio.cpp:60-147).
    iq: interleaved float (x-128)/128.  Per block A = M*24/125 - 1 = 2 949 audio samples (the
    reference writes floor(M*24/125) of the 2 950 its resampler yields, :226-229)."""
    co = mode1_coeffs(rf_taps)
    B = 2 * block_complex
    M = block_complex // 10
    A = M * 24 // 125
    zi_i, zi_q = np.zeros(rf_taps - 1), np.zeros(rf_taps - 1)
    phase = 0.0
    zr_m, zr_s = np.zeros(3622), np.zeros(3622)
    z_p, z_e = np.zeros(150), np.zeros(150)
    pll_state = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    out = []
    k = 0
    while (k + 1) * B <= len(iq) and (nblocks is None or k < nblocks):
        blk = iq[k * B:(k + 1) * B]
        i_f, zi_i = lfilter_fir(co["rf"], blk[0::2], zi_i)
        q_f, zi_q = lfilter_fir(co["rf"], blk[1::2], zi_q)
        dm, phase = fm_demod_arctan(i_f[::10], q_f[::10], phase)
        r = {"demod": dm}
        m, zr_m = resample(dm, co["res"], zr_m, 24, 125)
        r["pilot"], z_p = lfilter_fir(co["pilot"], dm, z_p)
        nco, _, pll_state = fm_pll(r["pilot"], 19e3, 250e3, list(pll_state), 2)
        r["nco"] = nco
        r["ext"], z_e = lfilter_fir(co["ext"], dm, z_e)
        mixed = nco[:M] * r["ext"] * 2
        s, zr_s = resample(mixed, co["res"], zr_s, 24, 125)
        r["audio"], r["stereo"] = m[:A], s[:A]
        r["left"] = (r["audio"] + r["stereo"]) / 2
        r["right"] = (r["audio"] - r["stereo"]) / 2
        out.append(r)
        k += 1
    return out


def rds_blocks(iq_u8, block_values=307200, taps=151, nblocks=None, demod_fn=fm_demod_arctan, pll_fn=fm_pll,
               alt_in=None, alt_from=0):
    """Restatement of model/fmRDSblock.py:127-204 (signal path up to the RRC filter).
    iq_u8: interleaved uint8, normalised (x-128)/128 as :59.  alt_in / alt_from: a second
    fmPll on the rows alt_in(k) (the device's own pre-PLL rows) and the mixer -> LPF ->
    resampler -> RRC statements after it, as mono_stereo_blocks' (r["alt"])."""
    iq = (np.asarray(iq_u8, dtype=np.float64) - 128.0) / 128.0
    rf_b, _ = mono_coeffs(taps, 151)
    co = rds_coeffs(taps)
    z = lambda: np.zeros(taps - 1)  # noqa: E731
    zi_i, zi_q, phase = z(), z(), 0.0
    ex_zi, sq_zi = z(), z()
    pll_state = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    phase_adj = math.pi / 3.3 - math.pi / 1.5

    def chain():
        return {"pll": list(pll_state), "li": z(), "lq": z(), "ai": z(), "aq": z(), "ri": np.zeros(150),
                "rq": np.zeros(150)}
    chains = [chain()] + ([chain()] if alt_in is not None else [])

    def rds_tail(r, c, x):
        nco_i, nco_q, c["pll"] = pll_fn(x, 114000, 240000, list(c["pll"]), ncoScale=0.5,
                                        phaseAdjust=phase_adj, normBandwidth=0.001)
        o = {"nco_i": nco_i, "nco_q": nco_q}
        if c is chains[0] or k >= alt_from - 1:
            n = len(r["extract"])
            o["lpf_i"], c["li"] = lfilter_fir(co["lpf"], np.multiply(r["extract"], nco_i[0:n]) * 2, c["li"])
            o["lpf_q"], c["lq"] = lfilter_fir(co["lpf"], np.multiply(r["extract"], nco_q[0:n]) * 2, c["lq"])
            o["resample_i"], c["ai"] = resample(o["lpf_i"], co["anti_img"], c["ai"], 19, 80)
            o["resample_q"], c["aq"] = resample(o["lpf_q"], co["anti_img"], c["aq"], 19, 80)
            o["rrc_i"], c["ri"] = lfilter_fir(co["rrc"], o["resample_i"], c["ri"])
            o["rrc_q"], c["rq"] = lfilter_fir(co["rrc"], o["resample_q"], c["rq"])
        return o
    out = []
    k = 0
    while (k + 1) * block_values < len(iq) and (nblocks is None or k < nblocks):   # :127
        blk = iq[k * block_values:(k + 1) * block_values]
        r = {}
        i_ds, zi_i = lfilter_decim(rf_b, blk[0::2], zi_i, 10)
        q_ds, zi_q = lfilter_decim(rf_b, blk[1::2], zi_q, 10)
        r["demod"], phase = demod_fn(i_ds, q_ds, phase)
        r["extract"], ex_zi = lfilter_fir(co["extract"], r["demod"], ex_zi)
        r["pre_pll"], sq_zi = lfilter_fir(co["square"], np.square(r["extract"]), sq_zi)
        r.update(rds_tail(r, chains[0], r["pre_pll"]))
        if alt_in is not None:
            r["alt"] = rds_tail(r, chains[1], np.asarray(alt_in(k), dtype=np.float64))
        out.append(r)
        k += 1
    return out


def mono_basic_coeffs(iq, rf_b, au_b, rf_decim=10, audio_decim=5, demod_fn=fm_demod_arctan):
    """model/fmMonoBasic.py:70-111 with given coefficients: returns (audio, demod)."""
    i_f = lfilter_fir(rf_b, iq[0::2])
    q_f = lfilter_fir(rf_b, iq[1::2])
    demod, _ = demod_fn(i_f[::rf_decim], q_f[::rf_decim], 0.0)
    return lfilter_fir(au_b, demod)[::audio_decim], demod


def mono_basic(iq, rf_taps=101, audio_taps=151, demod_fn=fm_demod_arctan):
    """Single-pass model/fmMonoBasic.py:67-136: lfilter without state over the whole
    capture, [::10], demod (prev 0), audio lfilter, [::5], int16(audio/2*32767)."""
    rf_b, au_b = mono_coeffs(rf_taps, audio_taps)
    i_f = lfilter_fir(rf_b, iq[0::2])
    q_f = lfilter_fir(rf_b, iq[1::2])
    demod, _ = demod_fn(i_f[::10], q_f[::10], 0.0)
    audio = lfilter_fir(au_b, demod)[::5]
    return audio, np.int16((audio / 2) * 32767)


# ---- RDS link layer ---------------------------------------------
# Parity matrix of model/fmRDSblock.py:49 (26 x 10) and the syndromes of :300-330.
RDS_H = np.array([[1,0,0,0,0,0,0,0,0,0],[0,1,0,0,0,0,0,0,0,0],[0,0,1,0,0,0,0,0,0,0],[0,0,0,1,0,0,0,0,0,0],
                  [0,0,0,0,1,0,0,0,0,0],[0,0,0,0,0,1,0,0,0,0],[0,0,0,0,0,0,1,0,0,0],[0,0,0,0,0,0,0,1,0,0],
                  [0,0,0,0,0,0,0,0,1,0],[0,0,0,0,0,0,0,0,0,1],[1,0,1,1,0,1,1,1,0,0],[0,1,0,1,1,0,1,1,1,0],
                  [0,0,1,0,1,1,0,1,1,1],[1,0,1,0,0,0,0,1,1,1],[1,1,1,0,0,1,1,1,1,1],[1,1,0,0,0,1,0,0,1,1],
                  [1,1,0,1,0,1,0,1,0,1],[1,1,0,1,1,1,0,1,1,0],[0,1,1,0,1,1,1,0,1,1],[1,0,0,0,0,0,0,0,0,1],
                  [1,1,1,1,0,1,1,1,0,0],[0,1,1,1,1,0,1,1,1,0],[0,0,1,1,1,1,0,1,1,1],[1,0,1,0,1,0,0,1,1,1],
                  [1,1,1,0,0,0,1,1,1,1],[1,1,0,0,0,1,1,0,1,1]], dtype=np.int64)
RDS_SYNDROMES = {0: [1,1,1,1,0,1,1,0,0,0], 1: [1,1,1,1,0,1,0,1,0,0],      # A, B
                 2: [1,0,0,1,0,1,1,1,0,0], 3: [1,0,0,1,0,1,1,0,0,0]}      # C, D


def rds_link(rrc_blocks):
    """Restatement of model/fmRDSblock.py:207-346 (clock and data recovery, Manchester and
    differential decoding, syndrome frame sync) over the per-block in-phase RRC outputs.
    Returns per block: symbols, bits, diff (the bits the syndrome scan sees, carried bits
    first) and events [(type 0..3 = A..D, position, accepted)], where accepted = the
    'Syndrome X at position' prints and not accepted = the 'False positive' prints.
    One deviation: a tie in the block-0 screening (:244-248 leaves start_pos unbound, a
    NameError) takes start_pos = 0."""
    out = []
    st = dict(block_count=0, int_offset=0, start_pos=0, lonely_bit=0.0, front_bit=0, prebit=0,
              printposition=0, prev_sync_bits=np.zeros(0), last_position=-1)
    for rrc in rrc_blocks:
        rrc = np.asarray(rrc, dtype=np.float64)
        r = {}
        if st["block_count"] == 0:                                             # :208-209
            st["int_offset"] = int(np.where(rrc[0:24] == np.max(rrc[0:24]))[0][0])
        io = st["int_offset"]
        s = rrc[io::24]                                                        # :216
        # :219 (value search in the last 24 samples; the value sits at a known index)
        st["int_offset"] = 24 - int(np.where(rrc[len(rrc) - 24:] == s[-1])[0][0])
        if st["block_count"] == 0:                                             # :233-249
            c0 = c1 = 0
            for m in range(int(len(s) / 4)):
                if (s[2 * m] > 0 and s[2 * m + 1] > 0) or (s[2 * m] < 0 and s[2 * m + 1] < 0):
                    c0 += 1
                elif (s[2 * m + 1] > 0 and s[2 * m + 2] > 0) or (s[2 * m + 1] < 0 and s[2 * m + 2] < 0):
                    c1 += 1
            st["start_pos"] = 1 if c0 > c1 else 0
        sp = st["start_pos"]
        bits = np.zeros(int(len(s) / 2) - sp)                                  # :251
        if sp == 1 and st["block_count"] != 0:                                 # :255-259
            if st["lonely_bit"] > s[0]:
                st["front_bit"] = 1
            elif st["lonely_bit"] < s[0]:
                st["front_bit"] = 0
        for k in range(len(bits)):                                             # :261-269
            if sp + 2 * k + 1 > len(s) - 1:
                break
            if s[2 * k + sp] > s[2 * k + 1 + sp]:
                bits[k] = 1
            elif s[2 * k + sp] < s[2 * k + 1 + sp]:
                bits[k] = 0
        if sp == 1:                                                            # :271-276
            bits = np.insert(bits, 0, st["front_bit"], axis=0)
            st["lonely_bit"] = s[-1]
        if st["block_count"] == 0:                                             # :280-284
            st["prebit"] = bits[0]
            off = 1
        else:
            off = 0
        diff = np.zeros(len(bits) - off)
        for t in range(len(diff)):                                             # :286-289
            pb, b = bool(st["prebit"]), bool(bits[t + off])
            diff[t] = (pb and not b) or (not pb and b)
            st["prebit"] = bits[t + off]
        st["prebit"] = bits[-1]                                                # :291
        if st["block_count"] != 0:                                             # :295-296
            diff = np.insert(diff, 0, st["prev_sync_bits"], axis=0)
        events = []
        position = 0
        while True:                                                            # :299-341
            blk = diff[position:position + 26].astype(np.int64)
            syn = ((blk @ RDS_H) % 2).tolist()
            for typ, pat in RDS_SYNDROMES.items():
                if syn == pat:
                    pp = st["printposition"]
                    if st["last_position"] == -1 or pp - st["last_position"] == 26:
                        events.append((typ, pp, 1))
                        st["last_position"] = pp
                    else:
                        events.append((typ, pp, 0))
                    break
            position += 1
            if position + 26 > len(diff) - 1:
                break
            st["printposition"] += 1
        st["prev_sync_bits"] = diff[position - 1:]                            # :343
        st["block_count"] += 1
        r.update(symbols=s, bits=bits, diff=diff, events=events)
        out.append(r)
    return out


# ---- spectral diagnostics --------------------------------------------
def estimate_psd(samples, nfft, fs):
    """Restatement of model/fmSupportLib.py:66-140 (estimatePSD): Bartlett estimate over
    floor(len/nfft) non-overlapping segments; Hann window pow(sin(i*pi/N), 2) (:80-82);
    np.fft.fft per segment (:101); 2 * (1/(Fs*N/2)) * |X_k|^2 for k < N/2 (:115-117);
    10*log10 per bin (:120-121, raises on a zero bin); dB averaged over segments in
    segment order (:128-137).  Returns (freq, psd_est)."""
    x = np.asarray(samples, dtype=np.float64)
    freq = np.arange(0, fs / 2, fs / nfft)
    hann = np.array([math.sin(i * math.pi / nfft) ** 2 for i in range(nfft)])
    nseg = len(x) // nfft
    half = nfft // 2
    rows = []
    for k in range(nseg):
        xf = np.fft.fft(x[k * nfft:(k + 1) * nfft] * hann, nfft)[:half]
        p = 2 * (1 / (fs * nfft / 2) * np.abs(xf) ** 2)
        if np.any(p <= 0):
            raise ValueError("math domain error")
        rows.append(10 * np.log10(p))
    est = np.zeros(half)
    for row in rows:
        est += row
    with np.errstate(invalid="ignore", divide="ignore"):
        return freq, est / nseg


def dft(x):
    """Restatement of model/fmSupportLib.py:46-60: X_m = sum_k x_k exp(i*2*pi*(-k*m)/N), the
    angle rounded as the reference's expression rounds it, summed in k order."""
    x = np.asarray(x, dtype=np.float64)
    n = len(x)
    k = np.arange(n, dtype=np.int64)
    out = np.zeros(n, dtype=np.complex128)
    for m in range(n):
        ang = (2 * math.pi) * (-k * m).astype(np.float64) / n
        terms = x * np.cos(ang) + 1j * (x * np.sin(ang))
        acc = 0j
        for t in terms:
            acc += t
        out[m] = acc
    return out
