"""Pin the CPU oracle (oracle/fm_oracle.py, oracle/fm_oracle.c) against the golden
vectors produced by the reference's own functions (tests/golden/make_golden.py).
CPU only."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from conftest import ROOT, maxabs

TIGHT = 1e-12


def test_golden_versions_recorded():
    import json
    v = json.load(open(os.path.join(ROOT, "tests", "golden", "VERSIONS.json")))
    assert v["numpy"] and v["scipy"] and "fmMonoBlock" not in v["generator"]


@pytest.mark.parametrize("taps", [101, 151])
def test_mono_stereo_loop_matches_golden(oracle, golden, taps):
    g = golden(f"mono_t{taps}.npz")
    iq = golden("mono_t101.npz")["iq"]
    B = int(g["block"][0])
    out = oracle.mono_stereo_blocks(iq, B, rf_taps=taps, stereo=(taps == 151))
    assert len(out) == g["demod"].shape[0] == 3
    for k, r in enumerate(out):
        for key in ("i_ds", "q_ds", "demod", "audio"):
            assert maxabs(r[key], g[key][k]) < 1e-11, (key, k)
        assert abs(r["phase"] - g["phase"][k][0]) < 1e-9
        if taps == 151:
            for key in ("bpf_recovery", "nco", "bpf_extraction", "stereo", "left", "right"):
                assert maxabs(r[key], g[key][k]) < 1e-10, (key, k)


def test_demod_loop_form_is_bit_exact_to_reference(oracle, golden):
    """The literal restatement reproduces the reference fmDemodArctan exactly."""
    g = golden("mono_t101.npz")
    d, p = oracle.fm_demod_arctan_loop(g["i_ds"][0], g["q_ds"][0], 0.0)
    assert np.array_equal(d, g["demod"][0])
    assert p == g["phase"][0][0]


def test_rds_chain_matches_golden(oracle, golden):
    g = golden("rds_u8.npz")
    out = oracle.rds_blocks(g["iq"], 307200)
    assert len(out) == 2
    for k, r in enumerate(out):
        for key in ("demod", "extract", "pre_pll", "nco_i", "nco_q", "lpf_i", "lpf_q",
                    "resample_i", "resample_q", "rrc_i", "rrc_q"):
            scale = max(1.0, float(np.max(np.abs(g[key][k]))))
            assert maxabs(r[key], g[key][k]) < 1e-9 * scale, (key, k)


@pytest.mark.parametrize("n", [1, 7, 149, 150, 151, 1000, 15360])
def test_decim_and_resample_fast_forms(oracle, n):
    """The checker's fast forms compute the literal statements' values: lfilter_decim ==
    lfilter_fir(...)[::D] with its zf (upfirdn, only the kept outputs), resample == the
    zero-stuffed lfilter (polyphase), on carried states, for short and long blocks."""
    rng = np.random.default_rng(n)
    x = rng.standard_normal(n)
    rf, au = oracle.mono_coeffs(151, 151)
    for b, D in ((rf, 10), (au, 5)):
        zi = rng.standard_normal(len(b) - 1)
        y, zf = oracle.lfilter_fir(b, x, zi)
        y2, zf2 = oracle.lfilter_decim(b, x, zi, D)
        assert y2.shape == y[::D].shape and maxabs(y2, y[::D]) < TIGHT and maxabs(zf2, zf) < TIGHT
    for b, up, down in ((oracle.rds_coeffs(151)["anti_img"], 19, 80), (oracle.mode1_coeffs()["res"], 24, 125)):
        zi = rng.standard_normal(len(b) - 1)
        y, zf = oracle.resample_literal(x, b, zi, up, down)
        y2, zf2 = oracle.resample(x, b, zi, up, down)
        assert y2.shape == y.shape and maxabs(y2, y) < TIGHT and maxabs(zf2, zf) < TIGHT


def test_oracle_alt_chain_is_the_chain(oracle, golden):
    """The second fmPll + downstream chain the span tests run on the device's loop inputs
    (alt_in / alt_from, tests/test_span.py): fed the oracle's own inputs, it reproduces the main
    chain -- the PLL bit for bit, every downstream row from block alt_from on (its filters start
    one block early from zero state) to rounding."""
    g = golden("mono_t151.npz")
    iq = golden("mono_t101.npz")["iq"]
    B = int(g["block"][0])
    base = oracle.mono_stereo_blocks(iq, B)
    out = oracle.mono_stereo_blocks(iq, B, alt_in=lambda k: base[k]["bpf_recovery"], alt_from=2)
    assert np.array_equal(out[0]["alt"]["nco"], out[0]["nco"]) and "stereo" not in out[0]["alt"]
    for k in (2,):
        for key in ("nco", "stereo", "left", "right"):
            assert maxabs(out[k]["alt"][key], out[k][key]) < TIGHT, (key, k)
    r = golden("rds_u8.npz")
    rb = oracle.rds_blocks(r["iq"], 307200)
    ro = oracle.rds_blocks(r["iq"], 307200, alt_in=lambda k: rb[k]["pre_pll"], alt_from=1)
    for k in range(len(ro)):
        for key in ("nco_i", "nco_q", "lpf_i", "lpf_q", "resample_i", "resample_q", "rrc_i", "rrc_q"):
            assert maxabs(ro[k]["alt"][key], ro[k][key]) < TIGHT, (key, k)


def test_mono_basic_matches_golden(oracle, golden):
    g = golden("basic_t101.npz")
    audio, wav = oracle.mono_basic(g["iq"], rf_taps=101)
    assert maxabs(audio, g["audio"]) < 1e-11
    assert np.array_equal(wav, g["wav"])


def test_demod_edge_cases(oracle, golden):
    u = golden("units.npz")
    for j in range(4):
        prev = float(u[f"demod{j}_prev_in"][0])
        for fn in (oracle.fm_demod_arctan, oracle.fm_demod_arctan_loop):
            d, p = fn(u["demod_I"], u["demod_Q"], prev)
            assert maxabs(d, u[f"demod{j}_d"]) < 1e-9
            assert abs(p - u[f"demod{j}_prev_out"][0]) < 1e-8


def test_lfilter_edge_cases(oracle, golden):
    u = golden("units.npz")
    from scipy import signal
    for taps in (101, 151):
        b = signal.firwin(taps, 0.1, window=("hann"))
        for n in (1, 7, 99, 150, 151, 1000, 5123):
            key = f"lf_t{taps}_n{n}"
            y, zf = oracle.lfilter_fir(b, u[key + "_x"], u[key + "_zi"])
            assert maxabs(y, u[key + "_y"]) < TIGHT
            assert maxabs(zf, u[key + "_zf"]) < TIGHT


def test_pll_chained_calls(oracle, golden):
    u = golden("units.npz")
    st = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    for j, (a, b) in enumerate(((0, 2500), (2500, 6000))):
        nco, ncoq, st = oracle.fm_pll(u["pll_in"][a:b], 19e3, 240e3, st, 2)
        assert maxabs(nco, u[f"pll{j}_nco"]) < 1e-12
        assert maxabs(ncoq, u[f"pll{j}_ncoq"]) < 1e-12
        assert maxabs(st, u[f"pll{j}_state"]) < 1e-9


def test_rrc_design(oracle, golden):
    u = golden("units.npz")
    assert maxabs(oracle.rrc_taps(57000, 151), u["rrc_57000_151"]) < 1e-15


def test_block_equals_single_pass(oracle, golden):
    """Known answer (spec p.4): block processing == single pass."""
    iq = golden("mono_t101.npz")["iq"][: 2 * 3 * 51200]
    blocks = oracle.mono_stereo_blocks(np.concatenate([iq, iq[:2]]), 51200, rf_taps=101, stereo=False)
    audio_b = np.concatenate([r["audio"] for r in blocks])
    rf_b, au_b = oracle.mono_coeffs(101, 151)
    i_f = oracle.lfilter_fir(rf_b, iq[0::2])[::10]
    q_f = oracle.lfilter_fir(rf_b, iq[1::2])[::10]
    d, _ = oracle.fm_demod_arctan(i_f, q_f, 0.0)
    audio_s = oracle.lfilter_fir(au_b, d)[::5]
    assert maxabs(audio_b, audio_s) < 1e-12


# ---- C restatement -------------------------------------------------------------------
@pytest.fixture(scope="module")
def liboracle():
    so = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    if not os.path.exists(so):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    lib = ctypes.CDLL(so)
    P = np.ctypeslib.ndpointer
    lib.orc_fir_decim.argtypes = [P(np.float32), ctypes.c_int64, ctypes.c_int64, P(np.float64), ctypes.c_int,
                                  ctypes.c_int, P(np.float64), P(np.float64)]
    lib.orc_demod.argtypes = [P(np.float64), P(np.float64), ctypes.c_int64, P(np.float64), P(np.float64)]
    lib.orc_fe_mono.argtypes = [P(np.float32), ctypes.c_int64, P(np.float64), ctypes.c_int, P(np.float64),
                                ctypes.c_int, P(np.float64), P(np.float64)]
    return lib


def test_c_oracle_lfilter(liboracle, golden):
    from scipy import signal
    u = golden("units.npz")
    for taps in (101, 151):
        b = np.ascontiguousarray(signal.firwin(taps, 0.1, window=("hann")))
        for n in (1, 7, 150, 1000, 5123):
            key = f"lf_t{taps}_n{n}"
            x = np.ascontiguousarray(u[key + "_x"], dtype=np.float32)
            zi = u[key + "_zi"].copy()
            y = np.empty(n)
            liboracle.orc_fir_decim(x, 1, n, b, taps, 1, zi, y)
            assert maxabs(y, u[key + "_y"]) < 1e-12
            assert maxabs(zi, u[key + "_zf"]) < 1e-12


def test_c_oracle_demod(liboracle, golden):
    u = golden("units.npz")
    for j in range(4):
        p = np.array([float(u[f"demod{j}_prev_in"][0])])
        out = np.empty(len(u["demod_I"]))
        liboracle.orc_demod(np.ascontiguousarray(u["demod_I"]), np.ascontiguousarray(u["demod_Q"]),
                            len(out), p, out)
        assert maxabs(out, u[f"demod{j}_d"]) < 1e-9
        assert abs(p[0] - u[f"demod{j}_prev_out"][0]) < 1e-8


def test_c_oracle_fe_mono(liboracle, golden, oracle):
    g = golden("basic_t101.npz")
    rf_b, au_b = oracle.mono_coeffs(101, 151)
    n = len(g["iq"]) // 2
    dm = np.empty((n + 9) // 10)
    au = np.empty(((n + 9) // 10 + 4) // 5)
    liboracle.orc_fe_mono(np.ascontiguousarray(g["iq"]), n, np.ascontiguousarray(rf_b), 101,
                          np.ascontiguousarray(au_b), 151, dm, au)
    assert maxabs(dm, g["demod"]) < 1e-11
    assert maxabs(au, g["audio"]) < 1e-11


def test_c_oracle_pll(oracle, golden):
    """orc_pll (oracle/fm_oracle.c) == fm_pll bit for bit -- the same restatement of
    model/fmPll.py:4-46 in C, used to run the oracle over hundreds of blocks
    (tests/test_span.py's bench-shape check) -- on the golden PLL fixture (chained calls,
    the stereo loop) and on the RDS loop's configuration (fmRDSblock.py:167)."""
    subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True, capture_output=True)
    u = golden("units.npz")
    x = u["pll_in"]
    for cfg in ((19e3, 240e3, 2.0, 0.0, 0.01), (114e3, 240e3, 0.5, np.pi / 3.3 - np.pi / 1.5, 0.001)):
        st_p, st_c = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0], [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
        for a, b in ((0, 700), (700, 1701), (1701, len(x))):
            ra = oracle.fm_pll(x[a:b], cfg[0], cfg[1], st_p, cfg[2], cfg[3], cfg[4])
            rb = oracle.fm_pll_c(x[a:b], cfg[0], cfg[1], st_c, cfg[2], cfg[3], cfg[4])
            assert np.array_equal(ra[0], rb[0]) and np.array_equal(ra[1], rb[1]) and ra[2] == rb[2]
            st_p, st_c = ra[2], rb[2]
    # and against the fixture itself (the reference's own fmPll, chained as test_pll_chained_calls)
    st = [0.0, 0.0, 1.0, 0.0, 1.0, 0.0]
    cuts = [0] + [len(u[f"pll{j}_nco"]) - 1 for j in range(2)]
    a = 0
    for j in range(2):
        b = a + cuts[j + 1]
        nco, ncoq, st = oracle.fm_pll_c(x[a:b], 19e3, 240e3, st, 2)
        assert maxabs(nco, u[f"pll{j}_nco"]) < 1e-12 and maxabs(ncoq, u[f"pll{j}_ncoq"]) < 1e-12
        a = b
