"""C-ABI boundary and host-side logic (CPU only: no compute call needs a GPU here)."""
import ctypes
import os
import re

import numpy as np
import pytest

from conftest import ROOT, maxabs

HEADER = os.path.join(ROOT, "include", "sdr.h")
LIB = os.path.join(ROOT, "real-time-software-defined-radio_amd", "libsdr.so")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(sdr_[a-z0-9_]+)\s*\(", text)))


def test_library_exports_every_declared_symbol():
    assert os.path.exists(LIB), "libsdr.so not built (run __graft_entry__.build())"
    lib = ctypes.CDLL(LIB)
    syms = header_symbols()
    assert len(syms) >= 25
    for s in syms:
        assert hasattr(lib, s), s


def test_ctypes_signatures_cover_header(sdr):
    from importlib import import_module
    _lib = import_module("real-time-software-defined-radio_amd._lib")
    assert sorted(_lib.SIGNATURES) == header_symbols()


def test_header_compiles_as_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "sdr.h"\nint main(void){return sdr_abi_version() == SDR_ABI_VERSION ? 0 : 1;}\n')
    import subprocess
    r = subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"), "-c",
                        str(src), "-o", str(tmp_path / "t.o")], capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


def test_abi_version_and_error_string(sdr):
    lib = sdr.load_library()
    assert lib.sdr_abi_version() == 1
    # a call that fails validation before touching any device
    rc = lib.sdr_create(0, None)
    assert rc == -1 and "NULL" in lib.sdr_last_error().decode()


def test_compute_fails_loudly_without_gpu(sdr):
    if sdr.device_count() > 0:
        pytest.skip("GPU present: covered by the gpu tests")
    with pytest.raises(sdr.SdrUnavailable):
        sdr.fmDemodArctan(np.ones(8), np.ones(8))
    with pytest.raises(sdr.SdrUnavailable):
        sdr.lfilter(np.ones(3) / 3, 1.0, np.ones(10), zi=np.zeros(2))


def test_argument_errors_mirror_scipy(sdr):
    """Shape/dtype errors are raised before any device work, like scipy's lfilter."""
    with pytest.raises(ValueError):
        sdr.lfilter(np.ones(5), 1.0, np.ones(10), zi=np.zeros(3))          # zi shape
    with pytest.raises(NotImplementedError):
        sdr.lfilter(np.ones(5), 1.0, np.ones(10, dtype=complex))             # complex
    with pytest.raises(NotImplementedError):
        sdr.lfilter(np.ones(5), [1.0, 0.5], np.ones(10))                     # IIR
    with pytest.raises(ValueError):
        sdr.rf_frontend_block(np.ones(7, np.float32), np.ones(5))            # odd interleaved length
    with pytest.raises(ValueError):
        sdr.fmPll(np.ones(4), 19e3, 240e3, [0.0] * 5)


def test_history_mapping_matches_reference_my_convoloution(sdr, golden, oracle):
    """my_convoloution's raw-history indexing (incl. the negative-index wrap) restated
    on the host, checked by running the FIR in the numpy oracle on [history, x]."""
    from importlib import import_module
    dsp = import_module("real-time-software-defined-radio_amd.dsp")
    u = golden("units.npz")
    h, x = u["myconv_h"], u["myconv_x"]
    for zi, y_ref in ((u["myconv_zw"], u["myconv_y1"]), (u["myconv_zfull"], u["myconv_y2"])):
        hist = dsp.history_from_my_zi(zi, len(h))
        y = oracle.lfilter_fir(h, np.concatenate([hist, x]))[len(hist):]
        assert maxabs(y, y_ref) < 1e-12
    with pytest.raises(IndexError):
        dsp.history_from_my_zi(np.zeros(5), 31)


def test_design_matches_reference(sdr, golden, oracle):
    u = golden("units.npz")
    assert maxabs(sdr.impulseResponseRootRaisedCosine(57000, 151), u["rrc_57000_151"]) < 1e-15
    assert maxabs(sdr.my_filterImpulseResponse(16e3, 240e3, 151), u["myfir_16k_240k_151"]) < 1e-15
    for a, b in zip(sdr.design.mono_coeffs(101, 151), oracle.mono_coeffs(101, 151)):
        assert np.array_equal(a, b)
    for a, b in zip(sdr.design.stereo_coeffs(), oracle.stereo_coeffs()):
        assert np.array_equal(a, b)
    ra, rb = sdr.design.rds_coeffs(), oracle.rds_coeffs()
    for k in ra:
        assert maxabs(ra[k], rb[k]) < 1e-15, k


def test_synthetic_iq_is_deterministic_and_bounded(sdr):
    a = sdr.synth.fm_iq(20000, seed=4)
    b = sdr.synth.fm_iq(20000, seed=4, chunk=3000)           # chunking does not change the stream
    assert a.dtype == np.float32 and a.shape == (40000,)
    assert np.array_equal(a, b)
    assert not np.array_equal(a, sdr.synth.fm_iq(20000, seed=5))
    u = sdr.synth.to_u8(a)
    assert u.dtype == np.uint8 and u.min() >= 0 and u.max() <= 255
    # per-IF-sample phase step stays below pi (no wrap ambiguity)
    z = a[0::2] + 1j * a[1::2]
    step = np.abs(np.angle(z[10::10] * np.conj(z[:-10:10])))
    assert np.percentile(step, 99) < np.pi


def test_product_never_imports_oracle():
    """The shipped package must not import, load or execute anything under oracle/."""
    import pathlib
    pkg = pathlib.Path(__file__).resolve().parents[1] / "real-time-software-defined-radio_amd"
    for f in list(pkg.rglob("*.py")) + list(pkg.rglob("*.hip")) + list(pkg.rglob("*.h")) + [pkg / "csrc" / "Makefile"]:
        text = f.read_text()
        assert "oracle" not in text.replace("never imports oracle", ""), f


def test_my_convoloution_empty_history_as_reference(sdr):
    """model/fmSupportLib.py:157-176 with my_zi = []: y[0] reads my_zi[-1] -> IndexError (any
    filter longer than one tap, non-empty block); an empty block reads nothing and returns
    x[-0:], i.e. the whole (empty) block, as the new state.  Both before any GPU work."""
    h = np.ones(5) / 5
    with pytest.raises(IndexError):
        sdr.my_convoloution(np.ones(8), h, 5, np.zeros(0))
    y, z = sdr.my_convoloution(np.zeros(0), h, 5, np.zeros(0))
    assert y.shape == (0,) and z.shape == (0,)
    y, z = sdr.my_convoloution(np.zeros(0), h, 5, np.arange(3.0))
    assert y.shape == (0,) and z.shape == (0,)          # x[-3:] of an empty block
