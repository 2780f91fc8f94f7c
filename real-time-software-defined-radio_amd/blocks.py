"""Device-resident block pipelines: the loops of model/fmMonoBlock.py and
model/fmRDSblock.py with every intermediate and every carried state in HBM.

Per block only the IQ block goes host->device and the requested outputs come back;
the filter states (lfilter zi, f64), the demod phase and the PLL state never leave
the GPU.  The stage order and the state threading follow the reference loops:

  MonoBlockProcessor    model/fmMonoBlock.py:86-109   
  StereoBlockProcessor  model/fmMonoBlock.py:113-173  (a9, a10; intended combiner)
  RdsBlockProcessor     model/fmRDSblock.py:133-204   (a9, a11; up to the RRC output)
"""
from __future__ import annotations

import numpy as np

from . import _lib
from . import design
from ._lib import SDR_IQ_F32, SDR_IQ_U8, SDR_PRE_MIX, SDR_PRE_NONE, SDR_PRE_SQUARE, DeviceBuffer, check, f64p
from .dsp import _taps


class _Filter:
    """One lfilter stage: taps (host f64, uploaded/cached by libsdr) + device zi."""

    def __init__(self, ctx, b):
        self.b = _taps(b)
        self.T = len(self.b)
        self.zi = DeviceBuffer(ctx, 8 * max(self.T - 1, 1))
        self.zi.zero()

    def run(self, ctx, x_ptr, n, y_ptr, decim=1, pre=SDR_PRE_NONE, mix_ptr=None, gain=1.0):
        check(ctx.lib.sdr_fir_dev(ctx.handle, x_ptr, mix_ptr, float(gain), int(pre), int(n), int(n), 0, 1,
                                  f64p(self.b), self.T, int(decim), self.zi.ptr, self.T - 1, self.zi.ptr,
                                  y_ptr, (n + decim - 1) // decim), "sdr_fir_dev")


class MonoBlockProcessor:
    """FE (RF LPF + decimate + atan2 demod) and mono audio LPF + decimate per block.

    block_complex: complex samples per block (model/fmMonoBlock.py:53 uses 51 200)."""

    def __init__(self, block_complex: int, rf_coeff=None, audio_coeff=None, rf_decim: int = 10,
                 audio_decim: int = 5, iq_dtype=np.float32, ctx=None):
        self.ctx = ctx if ctx is not None else _lib.get_context()
        if rf_coeff is None or audio_coeff is None:
            rc, ac = design.mono_coeffs()
            rf_coeff = rc if rf_coeff is None else rf_coeff
            audio_coeff = ac if audio_coeff is None else audio_coeff
        self.B = int(block_complex)
        self.rf_decim, self.audio_decim = int(rf_decim), int(audio_decim)
        self.u8 = np.dtype(iq_dtype) == np.uint8
        self.rf_b = _taps(rf_coeff)
        self.M = (self.B + self.rf_decim - 1) // self.rf_decim
        self.A = (self.M + self.audio_decim - 1) // self.audio_decim
        c = self.ctx
        self.iq = DeviceBuffer(c, self.B * (2 if self.u8 else 8))
        self.demod = DeviceBuffer(c, 4 * self.M + 16)
        self.audio = DeviceBuffer(c, 4 * self.A + 16)
        z = len(self.rf_b) - 1
        self.rf_state = DeviceBuffer(c, 8 * (2 * max(z, 1) + 1))  # zi_i | zi_q | phase
        self.rf_state.zero()
        self._z = max(z, 1)
        self.audio_f = _Filter(c, audio_coeff)

    def _frontend(self, iq_block):
        iq = np.ascontiguousarray(iq_block, dtype=np.uint8 if self.u8 else np.float32)
        if iq.shape[0] != 2 * self.B:
            raise ValueError(f"expected {2 * self.B} interleaved values, got {iq.shape[0]}")
        self.iq.upload(iq)
        c = self.ctx
        s = self.rf_state.ptr
        z = self._z
        check(c.lib.sdr_rf_frontend_dev(c.handle, self.iq.ptr, SDR_IQ_U8 if self.u8 else SDR_IQ_F32, self.B,
                                        self.B, 0, 1, f64p(self.rf_b), len(self.rf_b), self.rf_decim,
                                        s, s + 8 * z, z, s, s + 8 * z, s + 16 * z, self.demod.ptr, self.M,
                                        None, None), "sdr_rf_frontend_dev")

    def _mono(self):
        self.audio_f.run(self.ctx, self.demod.ptr, self.M, self.audio.ptr, self.audio_decim)

    def process(self, iq_block, return_demod: bool = False):
        """audio_block (float64) for one block [+ fm_demod]."""
        self._frontend(iq_block)
        self._mono()
        audio = self.audio.download(self.A).astype(np.float64)
        if return_demod:
            return audio, self.demod.download(self.M).astype(np.float64)
        return audio

    @property
    def phase(self) -> float:
        return float(self.rf_state.download(1, np.float64, offset=16 * self._z)[0])


class StereoBlockProcessor(MonoBlockProcessor):
    """Mono + stereo (model/fmMonoBlock.py:113-173, intended combiner L=(a+s)/2, R=(a-s)/2)."""

    def __init__(self, block_complex: int, rf_coeff=None, audio_coeff=None, stereo_taps: int = 151, **kw):
        super().__init__(block_complex, rf_coeff, audio_coeff, **kw)
        c = self.ctx
        pilot, band, lpf = design.stereo_coeffs(stereo_taps)
        self.pilot_f = _Filter(c, pilot)
        self.band_f = _Filter(c, band)
        self.lpf_f = _Filter(c, lpf)
        self.bpf_r = DeviceBuffer(c, 4 * self.M + 16)
        self.bpf_e = DeviceBuffer(c, 4 * self.M + 16)
        self.nco = DeviceBuffer(c, 4 * (self.M + 1) + 16)
        self.stereo = DeviceBuffer(c, 4 * self.A + 16)
        self.left = DeviceBuffer(c, 4 * self.A + 16)
        self.right = DeviceBuffer(c, 4 * self.A + 16)
        self.pll_state = DeviceBuffer.from_array(c, np.array([0.0, 0.0, 1.0, 0.0, 1.0, 0.0]))  # :76

    def process(self, iq_block, return_intermediates: bool = False):
        self._frontend(iq_block)
        self._mono()
        c, M = self.ctx, self.M
        self.pilot_f.run(c, self.demod.ptr, M, self.bpf_r.ptr)                         # :115-117
        check(c.lib.sdr_pll_dev(c.handle, self.bpf_r.ptr, M, M, 1, 19e3, 240e3, design.STEREO_PLL_SCALE, 0.0,
                                0.01, self.pll_state.ptr, self.nco.ptr, None, M + 1), "sdr_pll_dev")  # :119
        self.band_f.run(c, self.demod.ptr, M, self.bpf_e.ptr)                          # :150-151
        self.lpf_f.run(c, self.bpf_e.ptr, M, self.stereo.ptr, self.audio_decim,        # :155-162
                       pre=SDR_PRE_MIX, mix_ptr=self.nco.ptr, gain=2.0)
        check(c.lib.sdr_stereo_combine_dev(c.handle, self.audio.ptr, self.stereo.ptr, self.A, self.left.ptr,
                                           self.right.ptr), "combine")                # :166-170
        A = self.A
        out = dict(audio=self.audio.download(A), stereo=self.stereo.download(A),
                   left=self.left.download(A), right=self.right.download(A))
        if return_intermediates:
            out.update(demod=self.demod.download(M), bpf_recovery=self.bpf_r.download(M),
                       nco=self.nco.download(M + 1), bpf_extraction=self.bpf_e.download(M))
        return {k: v.astype(np.float64) for k, v in out.items()}


class RdsBlockProcessor(MonoBlockProcessor):
    """RDS signal path of model/fmRDSblock.py:156-204, from the demod stream to the RRC
    output (I and Q).  The bit-level link layer after :204 is out of scope."""

    def __init__(self, block_complex: int = 153600, rf_coeff=None, taps: int = 151, iq_dtype=np.uint8, **kw):
        super().__init__(block_complex, rf_coeff, None, iq_dtype=iq_dtype, **kw)
        c = self.ctx
        co = design.rds_coeffs(taps)
        self.extract_f = _Filter(c, co["extract"])
        self.square_f = _Filter(c, co["square"])
        self.lpf_i = _Filter(c, co["lpf"])
        self.lpf_q = _Filter(c, co["lpf"])
        self.anti_b = _taps(co["anti_img"])
        self.anti_zi_i = DeviceBuffer(c, 8 * (len(self.anti_b) - 1))
        self.anti_zi_q = DeviceBuffer(c, 8 * (len(self.anti_b) - 1))
        self.anti_zi_i.zero()
        self.anti_zi_q.zero()
        self.rrc_i = _Filter(c, co["rrc"])
        self.rrc_q = _Filter(c, co["rrc"])
        M = self.M
        self.R = (M * design.RDS_UP + design.RDS_DOWN - 1) // design.RDS_DOWN
        mk = lambda n: DeviceBuffer(c, 4 * n + 16)  # noqa: E731
        self.extract, self.pre_pll = mk(M), mk(M)
        self.nco_i, self.nco_q = mk(M + 1), mk(M + 1)
        self.lpf_out_i, self.lpf_out_q = mk(M), mk(M)
        self.res_i, self.res_q = mk(self.R), mk(self.R)
        self.rrc_out_i, self.rrc_out_q = mk(self.R), mk(self.R)
        self.pll_state = DeviceBuffer.from_array(c, np.array([0.0, 0.0, 1.0, 0.0, 1.0, 0.0]))  # :96

    def process(self, iq_block, return_intermediates: bool = False):
        self._frontend(iq_block)
        c, M, R = self.ctx, self.M, self.R
        self.extract_f.run(c, self.demod.ptr, M, self.extract.ptr)                                 # :156
        self.square_f.run(c, self.extract.ptr, M, self.pre_pll.ptr, pre=SDR_PRE_SQUARE)            # :161-164
        check(c.lib.sdr_pll_dev(c.handle, self.pre_pll.ptr, M, M, 1, design.RDS_PLL_FREQ, 240000.0,
                                design.RDS_PLL_SCALE, design.RDS_PHASE_ADJ, design.RDS_PLL_BW,
                                self.pll_state.ptr, self.nco_i.ptr, self.nco_q.ptr, M + 1), "sdr_pll_dev")  # :167
        self.lpf_i.run(c, self.extract.ptr, M, self.lpf_out_i.ptr, pre=SDR_PRE_MIX, mix_ptr=self.nco_i.ptr,
                       gain=2.0)                                                                     # :173,:180
        self.lpf_q.run(c, self.extract.ptr, M, self.lpf_out_q.ptr, pre=SDR_PRE_MIX, mix_ptr=self.nco_q.ptr,
                       gain=2.0)                                                                     # :175,:182
        for x, zi, y in ((self.lpf_out_i, self.anti_zi_i, self.res_i), (self.lpf_out_q, self.anti_zi_q, self.res_q)):
            check(c.lib.sdr_resample_dev(c.handle, x.ptr, M, f64p(self.anti_b), len(self.anti_b), design.RDS_UP,
                                         design.RDS_DOWN, zi.ptr, zi.ptr, y.ptr), "sdr_resample_dev")  # :184-199
        self.rrc_i.run(c, self.res_i.ptr, R, self.rrc_out_i.ptr)                                    # :202
        self.rrc_q.run(c, self.res_q.ptr, R, self.rrc_out_q.ptr)                                    # :204
        out = dict(rrc_i=self.rrc_out_i.download(R), rrc_q=self.rrc_out_q.download(R))
        if return_intermediates:
            out.update(demod=self.demod.download(M), extract=self.extract.download(M),
                       pre_pll=self.pre_pll.download(M), nco_i=self.nco_i.download(M + 1),
                       nco_q=self.nco_q.download(M + 1), lpf_i=self.lpf_out_i.download(M),
                       lpf_q=self.lpf_out_q.download(M), resample_i=self.res_i.download(R),
                       resample_q=self.res_q.download(R))
        return {k: v.astype(np.float64) for k, v in out.items()}


class RdsLinkLayer:
    """RDS link layer of model/fmRDSblock.py:207-346 on the host (libsdr C++, no GPU):
    clock and data recovery, Manchester and differential decoding, syndrome frame sync.

    process(rrc_i) takes one block of the in-phase RRC output (RdsBlockProcessor's
    'rrc_i') and returns dict(events=[(type, position, accepted)], symbols, bits, diff):
    type 0..3 = syndrome A..D, accepted = the reference's "Syndrome X at position N"
    prints (1) or its "False positive" prints (0); the state carries across calls."""

    TYPES = "ABCD"

    def __init__(self):
        import ctypes
        self._c = ctypes
        self.lib = _lib.load_library()
        h = ctypes.c_void_p()
        check(self.lib.sdr_rds_link_create(ctypes.byref(h)), "sdr_rds_link_create")
        self.handle = h

    def process(self, rrc_i):
        c = self._c
        x = np.ascontiguousarray(rrc_i, dtype=np.float64)
        n = len(x)
        ns_max = n // 24 + 2
        nb_max = ns_max // 2 + 2
        nd_max = nb_max + 64
        ev = np.empty(3 * (nd_max + 1), dtype=np.int64)
        sym = np.empty(ns_max)
        bits = np.empty(nb_max, dtype=np.uint8)
        diff = np.empty(nd_max, dtype=np.uint8)
        ne, ns, nb, nd = c.c_int64(), c.c_int64(), c.c_int64(), c.c_int64()
        vp = lambda a: a.ctypes.data_as(c.c_void_p)  # noqa: E731
        check(self.lib.sdr_rds_link_block(self.handle, f64p(x), n, vp(ev), nd_max + 1, c.byref(ne), vp(sym),
                                          ns_max, c.byref(ns), vp(bits), nb_max, c.byref(nb), vp(diff), nd_max,
                                          c.byref(nd)), "sdr_rds_link_block")
        events = [tuple(int(v) for v in ev[3 * k:3 * k + 3]) for k in range(ne.value)]
        return dict(events=events, symbols=sym[:ns.value].copy(), bits=bits[:nb.value].copy(),
                    diff=diff[:nd.value].copy())

    def close(self):
        if getattr(self, "handle", None):
            self.lib.sdr_rds_link_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
