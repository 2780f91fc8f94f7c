"""Time-parallel receiver spans (>= 256 device-resident blocks per stream):
a receiver whose block is K of the reference's 153 600-sample blocks processes the K blocks
of every stream in ONE chain of launches -- the FE and stage filters as one pass over the
span (block processing == a single pass, spec p.4), the PLLs as a long call
(pseudo-blocks solved in parallel and chained, csrc/pll.hip "long calls").

Checked against (a) the per-block receiver over the same K blocks (the reference's block
loop, model/fmRDSblock.py:127-204 and model/fmMonoBlock.py:80-173) and (b) the oracle, with
the PLL solver counters asserted (every pseudo-block solved in parallel)."""
import numpy as np
import pytest

from conftest import long_blocks, maxabs, rms
from test_receiver import AUDIO_MAX, AUDIO_RMS, RDS_TOL

pytestmark = pytest.mark.gpu

B5 = 153_600
NAMES = ["demod", "audio", "stereo", "left", "right", "bpf_recovery", "nco", "bpf_extraction"] + list(RDS_TOL)
NCO_NAMES = ("nco", "nco_i", "nco_q")
# span vs per-block receiver: the same f32 kernels; they differ only in how block starts are
# formed (lfilter zi added in f32 there, the continuous convolution here) and in the PLL's
# rounding (scan association): relative to each signal's peak
SPAN_REL = {"demod": 2e-6, "audio": 2e-6, "stereo": 2e-6, "left": 2e-6, "right": 2e-6,
            "bpf_recovery": 2e-6, "nco": 2e-7, "bpf_extraction": 2e-6, "extract": 2e-6, "pre_pll": 4e-6,
            "nco_i": 2e-7, "nco_q": 2e-7, "lpf_i": 4e-6, "lpf_q": 3e-5, "resample_i": 4e-6, "resample_q": 3e-5,
            "rrc_i": 4e-6, "rrc_q": 3e-5}


# A PLL's phase detector takes the sign of its input (model/fmPll.py:24-27), so where two correct
# computations of a loop's input (the span and the per-block VALU loop; f32 and the oracle's f64)
# round a sample within the rounding of zero to opposite sides, the two loops legitimately part for
# a while (a ~4e-3 NCO transient that decays within a block; an RDS I / Q row's window is taken
# relative to the I / Q pair's peak).  Such a FLIP is counted only where
# every sign-mismatched sample lies within FLIP_NEAR of zero (relative to the row's peak: the
# input rows' own tolerance) -- a wrong-sign sample any larger fails the test -- and at most
# FLIP_MAX per stream and comparison.  Blocks within FLIP_SPAN after a flip compare that loop's
# outputs at FLIP_REL (~2.5x the largest window measured, 5.9e-3), every other block at the tight
# tolerances.  The oracle checks do not rely on this: they also run the oracle's fmPll on the
# device's OWN loop inputs (identical signs, so no flip can occur) and the oracle's mixers and
# filters after it, and compare every block at the tight tolerances (_check_oracle_block).
FLIP_SPAN, FLIP_REL, FLIP_MAX = 3, 1.5e-2, 3
FLIP_NEAR = {"bpf_recovery": 2e-6, "pre_pll": 5e-6}
FLIP_DEPS = {"bpf_recovery": ("nco", "stereo", "left", "right"),
             "pre_pll": ("nco_i", "nco_q", "lpf_i", "lpf_q", "resample_i", "resample_q", "rrc_i", "rrc_q")}
# the device's NCO rows against the oracle's fmPll run on the device's own loop inputs: the f32
# rounding of the NCO value (<= 6e-8) plus, for the pilot loop's compact phase rows (sdr_nco.h,
# r06), the f32 rounding of a row's residual against its 32-step line -- <= 5e-8 rad while the
# loop acquires (|residual| up to ~0.3 rad, tools/th32_err.py), ~1e-8 once locked.  Measured:
# 1.11e-7 in block 0 of seed 70 (the acquisition), 3e-8 in the locked blocks.
NCO_REPLAY = 1.5e-7


def _flips(src, got, want):
    """True when `got` and `want` (one block of the loop input src) differ in sign anywhere;
    asserts that every such sample lies within FLIP_NEAR of zero"""
    bad = np.sign(got) != np.sign(want)
    if not np.any(bad):
        return False
    peak = max(float(np.max(np.abs(want))), 1e-3)
    far = float(np.max(np.abs(np.asarray(want, dtype=np.float64)[bad]))) / peak
    assert far <= FLIP_NEAR[src], (src, "a wrong-sign sample far from zero", far)
    return True


def _transient_blocks(row, tables, blocks, max_flips=FLIP_MAX):
    """{block k: the outputs inside a FLIP_SPAN window after a sign flip of their loop's input}
    between a span (row(src, k, n) = block k's n samples of output src) and per-block tables
    (tables[src][k][src]: the block loop's or the oracle's loop input), over `blocks` in order"""
    last = {src: -10 ** 9 for src in FLIP_DEPS}
    out, flips = {}, []
    for k in blocks:
        for src in FLIP_DEPS:
            want = tables[src][k][src]
            if _flips(src, row(src, k, len(want)), want):
                last[src] = k
                flips.append((src, k))
        out[k] = {nm for src, deps in FLIP_DEPS.items() if k - last[src] <= FLIP_SPAN for nm in deps}
    print("loop-input sign flips against the block tables (source, block):", flips)
    assert len(flips) <= max_flips, flips
    return out


def _oracle_blocks(oracle, iq_u8, nblk, rec, pre, alt_from=0):
    """The oracle's block loops (model/fmMonoBlock.py:80-173, model/fmRDSblock.py:127-204; fmPll
    by its C restatement, bit-identical to the Python one) over a u8 stream's first nblk
    blocks, each block also with r["alt"]: the oracle's fmPll run on the device's own loop
    inputs (rec(k): its bpf_recovery row, pre(k): its pre_pll row, block k) and the oracle's
    mixer / LPF / resampler / RRC / combiner after it"""
    f = (iq_u8.astype(np.float64) - 128.0) / 128.0
    mono = oracle.mono_stereo_blocks(f, B5, rf_taps=151, audio_taps=151, nblocks=nblk, pll_fn=oracle.fm_pll_c,
                                     alt_in=rec, alt_from=alt_from)
    rds = oracle.rds_blocks(iq_u8, 2 * B5, taps=151, nblocks=nblk, pll_fn=oracle.fm_pll_c, alt_in=pre,
                            alt_from=alt_from)
    return mono, rds


def _concat_blocks(rows, name):
    """per-block outputs (list over blocks of (S, n)) as one span row; NCO rows carry index 0
    = the previous block's last value, so block k contributes [0, M) and the last block M too"""
    if name in NCO_NAMES:
        return np.concatenate([r[:, :-1] for r in rows] + [rows[-1][:, -1:]], axis=1)
    return np.concatenate(rows, axis=1)


def test_span_receiver_equals_block_loop_and_oracle(sdr, gpu_ctx, oracle):
    S, K, spans = 2, 4, 2
    nblk = spans * K
    iq = np.stack([sdr.synth.fm_iq(nblk * B5 + 1, seed=70 + s, dtype=np.uint8) for s in range(S)])
    kw = dict(stereo=True, rds=True, iq_dtype=np.uint8)
    per_rx = sdr.Receiver(S, B5, **kw)
    per = [per_rx.process(iq[:, 2 * k * B5:2 * (k + 1) * B5], fetch=NAMES) for k in range(nblk)]
    span_rx = sdr.Receiver(S, K * B5, **kw)
    got = []
    for sp in range(spans):
        gpu_ctx.pll_stats(reset=True)
        got.append(span_rx.process(iq[:, 2 * sp * K * B5:2 * (sp + 1) * K * B5], fetch=NAMES))
        st = span_rx.pll_stats()
        print(f"span {sp} solver counters:", st)
        nb = long_blocks(K * (B5 // 10))
        assert st["recurrences"] == S * 2 * nb, st
        assert st["long_guessed"] + st["long_chained"] == S * 2 * nb, st
        # the first span starts at the stream start: the loops acquire over its first pseudo-blocks
        # (the RDS loop takes ~10 000 steps), which the sequential kernels may take -- how many
        # moves with the filters' rounding; the next span is locked and must be all parallel
        if sp > 0:
            assert st["sequential"] == 0, st

    def span_row(s):
        def row(src, k, n):
            sp, kk = divmod(k, K)
            return got[sp][src][s][kk * n:(kk + 1) * n]
        return row
    # span vs block loop, block by block (the loops' sign-flip windows at FLIP_REL)
    worst, loose = {}, {}
    for s in range(S):
        tables = {src: {k: {src: per[k][src][s]} for k in range(nblk)} for src in FLIP_DEPS}
        trans = _transient_blocks(span_row(s), tables, range(nblk), FLIP_MAX)
        for name in NAMES:
            scale = max(max(float(np.max(np.abs(per[k][name][s]))) for k in range(nblk)), 1e-3)
            for k in range(nblk):
                sp, kk = divmod(k, K)
                w = per[k][name][s]
                n = len(w) - 1 if name in NCO_NAMES else len(w)
                g = got[sp][name][s][kk * n:kk * n + len(w)]
                assert g.shape == w.shape, (name, k)
                tgt = loose if name in trans[k] else worst
                tgt[name] = max(tgt.get(name, 0.0), maxabs(g, w) / scale)
    print("span vs block loop, max error relative to peak:", {k: f"{v:.1e}" for k, v in worst.items()},
          "; sign-flip windows:", {k: f"{v:.1e}" for k, v in loose.items()})
    for name in NAMES:
        assert worst.get(name, 0.0) < SPAN_REL[name], (name, worst[name])
        assert loose.get(name, 0.0) < FLIP_REL, (name, loose[name])
    # the span's carried states continue the block loop's
    for a, b in zip(span_rx.state(), per_rx.state()):
        assert maxabs(a, b) < 1e-6
    # against the oracle (stream 0, every block; the loops also on the span's own inputs)
    M = B5 // 10
    dev = lambda src: lambda k: span_row(0)(src, k, M)   # noqa: E731
    mono, rds = _oracle_blocks(oracle, iq[0], nblk, dev("bpf_recovery"), dev("pre_pll"))
    trans = _transient_blocks(span_row(0), {"bpf_recovery": mono, "pre_pll": rds}, range(nblk))
    errs = {}
    for k in range(nblk):
        sp, kk = divmod(k, K)
        g = got[sp]
        _check_oracle_block(lambda key: g[key][0], kk, mono[k], rds[k], trans[k], (k,), errs)
    _print_errs(errs)


def test_span_bench_shape_matches_block_loop_and_oracle(sdr, gpu_ctx, oracle):
    """The exact shape bench.py's c5_1stream leg times: ONE u8 stream, spans of K = 256 blocks
    (3.9 M PLL steps per recurrence: 275 pseudo-blocks chained, the RDS loop's linear
    acceptance and the NCO's linear response over the whole span), two spans in a row.
    Checked against (a) the per-block receiver over all 512 blocks (the reference's block
    loop) at SPAN_REL, and (b) the oracle (model/fmMonoBlock.py:80-173,
    model/fmRDSblock.py:127-204, run over all 512 blocks with the C restatement of fmPll,
    bit-identical to the Python one) on every block, its loops also run on the span's own
    inputs (_check_oracle_block); the solver counters of the locked span: every pseudo-block solved in parallel in round 0, no
    chain stop, no sequential tail."""
    K, spans = 256, 2
    nblk = K * spans
    iq = sdr.synth.fm_iq(nblk * B5 + 1, seed=7, dtype=np.uint8)[None, :]
    kw = dict(stereo=True, rds=True, iq_dtype=np.uint8)
    span_rx = sdr.Receiver(1, K * B5, **kw)
    nb = long_blocks(K * (B5 // 10))
    got, stats = [], []
    for sp in range(spans):
        gpu_ctx.pll_stats(reset=True)
        got.append(span_rx.process(iq[:, 2 * sp * K * B5:2 * (sp + 1) * K * B5], fetch=NAMES))
        stats.append(span_rx.pll_stats())
        print(f"span {sp} (K={K}) solver counters:", stats[-1])
    for sp, st in enumerate(stats):
        assert st["recurrences"] == 2 * nb and st["long_tail"] == 0, (sp, st)
    st = stats[1]
    assert st["spec_r0"] == 2 * nb and st["sequential"] == 0 and st["long_stops"] == 0, st
    # (a) the per-block receiver over every block of both spans
    per_rx = sdr.Receiver(1, B5, **kw)
    M = B5 // 10
    peak, worst, loose = {}, {}, {}
    last_flip = {src: -10 ** 9 for src in FLIP_DEPS}
    flips = []
    for k in range(nblk):
        p = per_rx.process(iq[:, 2 * k * B5:2 * (k + 1) * B5], fetch=NAMES)
        sp, kk = divmod(k, K)
        blk = {}
        for name in NAMES:
            w = p[name][0]
            n = len(w) - 1 if name in NCO_NAMES else len(w)
            g = got[sp][name][0][kk * n:kk * n + len(w)]
            assert g.shape == w.shape, (name, k)
            blk[name] = (g, w)
            peak[name] = max(peak.get(name, 0.0), float(np.max(np.abs(w))))
        for src in FLIP_DEPS:
            if _flips(src, *blk[src]):
                last_flip[src] = k
                flips.append((src, k))
        for name in NAMES:
            g, w = blk[name]
            transient = any(name in deps and k - last_flip[src] <= FLIP_SPAN for src, deps in FLIP_DEPS.items())
            tgt = loose if transient else worst
            tgt[name] = max(tgt.get(name, 0.0), maxabs(g, w))
    rel = {name: worst.get(name, 0.0) / max(peak[name], 1e-3) for name in NAMES}
    print("bench-shape span vs block loop, max error relative to peak:", {k: f"{v:.1e}" for k, v in rel.items()})
    print("loop-input sign flips (source, block):", flips, "; their windows:",
          {k: f"{v / max(peak[k], 1e-3):.1e}" for k, v in loose.items()})
    assert len(flips) <= FLIP_MAX, flips
    for name in NAMES:
        assert rel[name] < SPAN_REL[name], (name, rel[name])
        assert loose.get(name, 0.0) / max(peak[name], 1e-3) < FLIP_REL, (name, loose[name])
    for a, b in zip(span_rx.state(), per_rx.state()):
        assert maxabs(a, b) < 1e-6
    del per_rx

    # (b) the oracle on every block of both spans, its loops also run on the span's own inputs
    def span_row(src, k, n):
        sp, kk = divmod(k, K)
        return got[sp][src][0][kk * n:(kk + 1) * n]
    dev = lambda src: lambda k: span_row(src, k, M)    # noqa: E731
    mono, rds = _oracle_blocks(oracle, iq[0], nblk, dev("bpf_recovery"), dev("pre_pll"))
    trans = _transient_blocks(span_row, {"bpf_recovery": mono, "pre_pll": rds}, range(nblk))
    errs = {}
    for k in range(nblk):
        sp, kk = divmod(k, K)
        g = got[sp]
        _check_oracle_block(lambda key: g[key][0], kk, mono[k], rds[k], trans[k], (k,), errs)
    _print_errs(errs)


def _check_oracle_block(row, kk, mono_k, rds_k, trans, tag, errs):
    """block kk of a span's outputs (row(key): the span row) against the oracle's block:
      (a) every output upstream of the PLLs (demod, audio, the loops' inputs bpf_recovery /
          pre_pll, bpf_extraction, extract) against the oracle's own rows;
      (b) the NCO rows against the oracle's fmPll run on the device's own loop inputs
          (mono_k["alt"], rds_k["alt"]: same signs, so no flip) at NCO_REPLAY;
      (c) everything downstream of the PLLs against the oracle's mixers and filters after that
          NCO, at the tight tolerances;
      (d) end to end against the oracle's own chain: the outputs in `trans` (a loop-input sign-
          flip window) at FLIP_REL of their peak, the others as (b) / (c).
    errs: the worst error per (check, output), updated"""
    A, M = len(mono_k["audio"]), len(mono_k["nco"]) - 1

    def note(key, v):
        errs[key] = max(errs.get(key, 0.0), v)

    def seg(key, want):
        n = len(want) - 1 if key in NCO_NAMES else len(want)
        gv = row(key)[kk * n:kk * n + len(want)]
        assert gv.shape == want.shape, (key,) + tag
        return gv

    def audio_ok(key, gv, want, chk):
        r, m = rms(gv, want), maxabs(gv, want)
        note((chk, key), m)
        assert r < AUDIO_RMS and m < AUDIO_MAX, (chk, key, r, m) + tag

    def rds_ok(key, gv, want, chk):
        tmax, trms = RDS_TOL[key]
        scale = max(float(np.max(np.abs(want))), 1e-3)
        em, er = maxabs(gv, want) / scale, rms(gv, want) / scale
        note((chk, key), em)
        assert em < tmax and er < trms, (chk, key, em, er) + tag

    def flip_ok(key, gv, want):
        # an RDS I or Q row relative to the pair's peak (one complex signal: the loop's transient
        # moves both by about the same amount, and Q is small next to I once locked)
        pair = {"_i": "_q", "_q": "_i"}.get(key[-2:])
        peak = float(np.max(np.abs(want)))
        if pair is not None:
            peak = max(peak, float(np.max(np.abs(rds_k[key[:-2] + pair]))))
        e = maxabs(gv, want) / max(peak, 1e-3)
        note(("flip", key), e)
        assert e < FLIP_REL, ("flip window", key, e) + tag
    # (a) upstream of the loops
    for key in ("demod", "audio"):
        audio_ok(key, seg(key, mono_k[key]), mono_k[key], "a")
    for key, tol in (("bpf_recovery", 2e-6), ("bpf_extraction", 4e-6)):      # relative to the peak
        want = mono_k[key]
        m = maxabs(seg(key, want), want) / max(float(np.max(np.abs(want))), 1e-3)
        note(("a", key), m)
        assert m < tol, ("a", key, m) + tag
    for key in ("extract", "pre_pll"):
        rds_ok(key, seg(key, rds_k[key]), rds_k[key], "a")
    # (b) the loops on the device's own inputs, (c) what follows them
    for key, alt in (("nco", mono_k["alt"]), ("nco_i", rds_k["alt"]), ("nco_q", rds_k["alt"])):
        m = maxabs(seg(key, alt[key]), alt[key])
        note(("b", key), m)
        assert m < NCO_REPLAY, ("b", key, m) + tag
    for key in ("stereo", "left", "right"):
        audio_ok(key, seg(key, mono_k["alt"][key]), mono_k["alt"][key], "c")
    for key in ("lpf_i", "lpf_q", "resample_i", "resample_q", "rrc_i", "rrc_q"):
        rds_ok(key, seg(key, rds_k["alt"][key]), rds_k["alt"][key], "c")
    # (d) end to end
    for key in ("stereo", "left", "right"):
        want = mono_k[key]
        flip_ok(key, seg(key, want), want) if key in trans else audio_ok(key, seg(key, want), want, "d")
    for key in ("nco", "nco_i", "nco_q"):
        want = (mono_k if key == "nco" else rds_k)[key]
        if key in trans:
            flip_ok(key, seg(key, want), want)
        else:
            m = maxabs(seg(key, want), want)
            note(("d", key), m)
            assert m < NCO_REPLAY, ("d", key, m) + tag
    for key in ("lpf_i", "lpf_q", "resample_i", "resample_q", "rrc_i", "rrc_q"):
        want = rds_k[key]
        flip_ok(key, seg(key, want), want) if key in trans else rds_ok(key, seg(key, want), want, "d")


def _print_errs(errs):
    print("span vs oracle, worst error per (check, output) -- a: upstream, b: NCO on the device's loop "
          "inputs, c: downstream of that NCO, d: end to end, flip: sign-flip windows:",
          {f"{c}:{k}": f"{v:.1e}" for (c, k), v in sorted(errs.items())})


def test_span_c5_timed_shape_eight_streams(sdr, gpu_ctx, oracle):
    """The exact shape and path bench.py's `c5` line times: EIGHT u8
    streams in one receiver, spans of K = 256 blocks from device memory (sdr_rx_process_dev),
    i.e. a PLL job table of 16 recurrences x 275 pseudo-blocks chained in one launch, with the
    bench's keep set (no NCO or RDS LPF rows: the mixers form the NCO from the PLL phases, the
    RDS LPF runs inside the composite resampler; no f32 PLL-input rows: the PLLs read sign
    codes).  Two spans of a continuous stream per stream
    (the second is the locked, timed state); the 8 streams are distinct windows of one
    synthetic capture.  Checked:
      (a) stream s of the 8-stream lean span == a 1-stream span over the same IQ that
          materialises every intermediate, bit for bit, for every output both produce (the
          streams of a job table are independent; the NCO formed in the mixers is the NCO row);
      (b) streams 0 and 7 against the oracle (model/fmMonoBlock.py:80-173,
          model/fmRDSblock.py:127-204 with the C restatement of fmPll) on every block of the
          second span, the intermediates from the 1-stream receiver, the oracle's loops also
          run on the receiver's own loop inputs (_check_oracle_block);
      (c) the solver counters: 16 x 275 recurrences per span, no sequential tail; the locked
          span all in round 0, no chain stop."""
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")
    S, K, spans = 8, 256, 2
    n = K * B5
    delta = 1_000_050                                   # window offset between streams (x 50: whole audio samples)
    base = sdr.synth.fm_iq(spans * n + (S - 1) * delta + 1, seed=91, dtype=np.uint8)
    win = lambda s: base[2 * s * delta:2 * (s * delta + spans * n + 1)]   # noqa: E731  (+1: the oracle's strict <)
    rows = np.ascontiguousarray(np.stack([win(s)[:2 * spans * n] for s in range(S)]))
    d = _lib.DeviceBuffer.from_array(gpu_ctx, rows)
    row_bytes = rows.shape[1]
    del rows
    kw = dict(stereo=True, rds=True, iq_dtype=np.uint8)
    lean = [nm for nm in NAMES if nm not in NCO_NAMES + ("lpf_i", "lpf_q", "bpf_recovery", "pre_pll")]
    rx = sdr.Receiver(S, n, keep=lean, **kw)
    nb = long_blocks(K * (B5 // 10))
    stats = []
    for sp in range(spans):
        gpu_ctx.pll_stats(reset=True)
        rx.process_dev(d.ptr + sp * 2 * n, spans * n)     # stride: the row of every stream
        stats.append(rx.pll_stats())
        print(f"S8 span {sp} solver counters:", stats[-1])
    for sp, st in enumerate(stats):
        assert st["recurrences"] == 2 * S * nb and st["long_tail"] == 0, (sp, st)
    st = stats[-1]
    assert st["spec_r0"] == 2 * S * nb and st["sequential"] == 0 and st["long_stops"] == 0, st
    got = {name: rx.output(name) for name in lean}
    for name in ("nco_i", "pre_pll", "bpf_recovery"):
        with pytest.raises(ValueError, match="not materialised"):
            rx.output(name)
    rx.close()
    # (a) every stream against a 1-stream receiver over the same two spans, every output kept
    one = sdr.Receiver(1, n, **kw)
    full, first = {}, {}
    for s in range(S):
        one.reset()
        for sp in range(spans):
            one.process_dev(d.ptr + s * row_bytes + sp * 2 * n, n)
            if sp == 0 and s in (0, S - 1):          # the first span's loop inputs (the replayed loops' state)
                first[s] = {src: one.output(src)[0].copy() for src in FLIP_DEPS}
        for name in lean:
            assert np.array_equal(one.output(name)[0], got[name][s]), (name, s)
        if s in (0, S - 1):
            full[s] = {name: one.output(name)[0] for name in NAMES}
    one.close()
    d.free()
    # (b) streams 0 and 7 against the oracle on every block of the second span, the loops also on
    # the receiver's own inputs (from the stream start: the loops' state)
    M = B5 // 10
    for s in (0, S - 1):
        g = full[s]
        rows = lambda src: lambda k: (first[s] if k < K else g)[src][(k % K) * M:(k % K + 1) * M]   # noqa: E731
        mono, rds = _oracle_blocks(oracle, win(s), spans * K, rows("bpf_recovery"), rows("pre_pll"), alt_from=K)
        # (the sign-flip windows over both spans: the first span's inputs are held too)
        trans = _transient_blocks(lambda src, k, n: rows(src)(k), {"bpf_recovery": mono, "pre_pll": rds},
                                  range(spans * K))
        errs = {}
        for kk in range(K):
            k = K + kk
            _check_oracle_block(lambda key: g[key], kk, mono[k], rds[k], trans[k], (s, k), errs)
        _print_errs(errs)
        del mono, rds


def test_span_mixers_equal_their_nco_rows(sdr, gpu_ctx, oracle):
    """The span's mixers form their NCO from the PLL's compact phase rows (sdr_nco.h, r06) --
    the stereo mixer on the matrix cores, the kept RDS LPF rows on the VALU tiles -- instead of
    reading NCO rows.  Pinned against the NCO rows the NCO kernel writes from the same phases
    (materialised here): the reference's mixer + LPF statements (model/fmMonoBlock.py:155-162,
    model/fmRDSblock.py:173-182) run on the host over those rows and the device's own mixer
    inputs reproduce the device's stereo and RDS LPF rows."""
    K = 4
    iq = sdr.synth.fm_iq(K * B5 + 1, seed=71, dtype=np.uint8)[None, :]
    rx = sdr.Receiver(1, K * B5, stereo=True, rds=True, iq_dtype=np.uint8)
    names = ["nco", "bpf_extraction", "stereo", "nco_i", "nco_q", "extract", "lpf_i", "lpf_q"]
    got = rx.process(iq[:, :2 * K * B5], fetch=names)
    g = {k: np.asarray(got[k][0], dtype=np.float64) for k in names}
    n = len(g["bpf_extraction"])
    _, _, st_b = oracle.stereo_coeffs(151)
    lpf = oracle.rds_coeffs(151)["lpf"]
    stereo, _ = oracle.lfilter_decim(st_b, g["nco"][:n] * g["bpf_extraction"] * 2, np.zeros(150), 5)
    lpf_i, _ = oracle.lfilter_fir(lpf, g["extract"] * g["nco_i"][:n] * 2, np.zeros(150))
    lpf_q, _ = oracle.lfilter_fir(lpf, g["extract"] * g["nco_q"][:n] * 2, np.zeros(150))
    errs = {}
    for name, want in (("stereo", stereo), ("lpf_i", lpf_i), ("lpf_q", lpf_q)):
        assert g[name].shape == want.shape, name
        errs[name] = maxabs(g[name], want) / max(float(np.max(np.abs(want))), 1e-3)
    print("mixers vs their NCO rows, max error relative to peak:", {k: f"{v:.1e}" for k, v in errs.items()})
    # (measured 2.9e-7 / 4.3e-7 / 2.0e-7: the mixers' f32 cos / sin against the rows' f64 ones
    # rounded to f32, and f32 mixing against the host's f64)
    for name, tol in (("stereo", 1e-6), ("lpf_i", 2e-6), ("lpf_q", 1e-6)):
        assert errs[name] < tol, (name, errs[name])


@pytest.mark.parametrize("K", [1, 4])
def test_keep_lean_equals_full(sdr, gpu_ctx, K):
    """sdr_rx_set_keep without the NCO and RDS LPF rows (the bench's receivers): every output
    both receivers produce is bit-identical to the receiver that materialises everything --
    per-block (K = 1: the solve's phases) and spans (K = 4: long calls, the chain's turns and
    linear responses applied in the mixers) -- over 3 calls, and so are the carried states."""
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")
    S, calls = 3, 3
    n = K * B5
    iq = np.stack([sdr.synth.fm_iq(calls * n, seed=120 + s, dtype=np.uint8) for s in range(S)])
    d = _lib.DeviceBuffer.from_array(gpu_ctx, iq)
    kw = dict(stereo=True, rds=True, iq_dtype=np.uint8)
    lean_names = [nm for nm in NAMES if nm not in NCO_NAMES + ("lpf_i", "lpf_q", "bpf_recovery", "pre_pll")]
    full, lean = sdr.Receiver(S, n, **kw), sdr.Receiver(S, n, keep=lean_names, **kw)
    for k in range(calls):
        for rx in (full, lean):
            rx.process_dev(d.ptr + 2 * k * n, calls * n)
        for name in lean_names:
            assert np.array_equal(lean.output(name), full.output(name)), (name, k)
    for a, b in zip(lean.state(), full.state()):
        assert np.array_equal(a, b)
    d.free()
