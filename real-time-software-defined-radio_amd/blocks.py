"""Device-resident block pipelines: the loops of model/fmMonoBlock.py and
model/fmRDSblock.py with every intermediate and every carried state in HBM.

All of them run on libsdr's multi-stream block receiver (sdr_rx_*, csrc/rx.hip): one
block of S independent streams is a fixed chain of ~10 launches -- the RF front end, one
launch per filter stage for all of that stage's filters and their lfilter final states,
and one lane per PLL recurrence -- whatever S is.  Per block only the IQ goes
host->device and the requested outputs come back; filter states (lfilter zi, f64), demod
phases and PLL states never leave the GPU.  Stage order and state threading follow the
reference loops:

  Receiver              S streams of any of the below at once
  MonoBlockProcessor    model/fmMonoBlock.py:86-109   
  StereoBlockProcessor  model/fmMonoBlock.py:113-173  (a9, a10; intended combiner)
  RdsBlockProcessor     model/fmRDSblock.py:133-204   (a9, a11; up to the RRC output)
"""
from __future__ import annotations

import collections
import ctypes

import numpy as np

from . import _lib
from . import design
from ._lib import RX_FILTERS, RX_OUTPUTS, SDR_IQ_F32, SDR_IQ_U8, SDR_RX_AUDIO, SDR_RX_RDS, SDR_RX_STEREO, check, f64p
from .dsp import _taps

_PLL_INIT = (0.0, 0.0, 1.0, 0.0, 1.0, 0.0)       # model/fmMonoBlock.py:76, model/fmRDSblock.py:96


def _addr(a):
    """The data address of a C-contiguous array: a writable one through the buffer protocol
    (~0.6 us), anything else through ndarray.ctypes (~1.5-2 us, a ctypes object per call).
    At the reference's block sizes a block costs ~30-45 us, so per-call pointer lookups show."""
    if a.flags.writeable and a.nbytes:
        return ctypes.addressof(ctypes.c_char.from_buffer(a))
    return a.ctypes.data


class Receiver:
    """`nstreams` independent FM streams through the block receiver (sdr_rx).

    Each call to process() takes one block of every stream: an (nstreams, 2*block) array of
    interleaved IQ (f32, or u8 as read from rtl_sdr, src/iofunc.cpp:61-69).  mono=True
    produces the mono audio (model/fmMonoBlock.py:86-109); stereo=True adds the pilot PLL,
    the stereo channel and L/R (:113-173); rds=True the RDS chain to the RRC output
    (model/fmRDSblock.py:156-204).  Outputs (output(), process()'s return) are float32
    arrays of shape (nstreams, n); names as in the reference loops ("audio", "stereo",
    "left", "right", "rrc_i", ...: _lib.RX_OUTPUTS)."""

    def __init__(self, nstreams: int, block_complex: int, *, mono: bool = True, stereo: bool = False,
                 rds: bool = False, iq_dtype=np.uint8, rf_coeff=None, audio_coeff=None, stereo_taps: int = 151,
                 rds_taps: int = 151, rf_decim: int = 10, audio_decim: int = 5, pipeline: bool = False,
                 depth: int = 1, keep=None, ctx=None):
        self.ctx = ctx if ctx is not None else _lib.get_context()
        self.lib = self.ctx.lib
        self.S, self.B = int(nstreams), int(block_complex)
        self.u8 = np.dtype(iq_dtype) == np.uint8
        flags = (SDR_RX_AUDIO if mono else 0) | (SDR_RX_STEREO if stereo else 0) | (SDR_RX_RDS if rds else 0)
        self.flags = flags
        self._lengths = {}
        self._plans = {}
        self._pending = collections.deque()   # submit(): the blocks in flight's output arrays
        self.depth = int(depth)
        h = ctypes.c_void_p()
        check(self.lib.sdr_rx_create(self.ctx.handle, self.S, self.B, SDR_IQ_U8 if self.u8 else SDR_IQ_F32,
                                     flags, ctypes.byref(h)), "sdr_rx_create")
        self.handle = h
        if pipeline:                          # front half of block k+1 beside the back half of k
            check(self.lib.sdr_rx_set_pipeline(self.handle, 1), "sdr_rx_set_pipeline")
        if self.depth != 1:                   # submit(): `depth` blocks in flight
            check(self.lib.sdr_rx_set_depth(self.handle, self.depth), "sdr_rx_set_depth")
        if rf_coeff is None or audio_coeff is None:
            rc, ac = design.mono_coeffs()
            rf_coeff = rc if rf_coeff is None else rf_coeff
            audio_coeff = ac if audio_coeff is None else audio_coeff
        taps = {"rf": rf_coeff, "audio": audio_coeff}
        if stereo:
            taps.update(zip(("pilot", "stereo_bpf", "stereo_lpf"), design.stereo_coeffs(stereo_taps)))
        if rds:
            co = design.rds_coeffs(rds_taps)
            taps.update(rds_extract=co["extract"], rds_square=co["square"], rds_lpf=co["lpf"],
                        rds_anti=co["anti_img"], rds_rrc=co["rrc"])
        for name, b in taps.items():
            b = _taps(b)
            check(self.lib.sdr_rx_set_filter(self.handle, RX_FILTERS.index(name), f64p(b), len(b)),
                  "sdr_rx_set_filter")
        check(self.lib.sdr_rx_set_decim(self.handle, int(rf_decim), int(audio_decim), design.RDS_UP,
                                        design.RDS_DOWN), "sdr_rx_set_decim")
        if keep is not None:
            self.set_keep(keep)
        self.M = (self.B + rf_decim - 1) // rf_decim
        self.A = (self.M + audio_decim - 1) // audio_decim
        self.R = (self.M * design.RDS_UP + design.RDS_DOWN - 1) // design.RDS_DOWN

    @property
    def outputs(self):
        """Names of the outputs this configuration produces."""
        return [n for k, n in enumerate(RX_OUTPUTS) if self._produces(k)]

    def _produces(self, k):
        name = RX_OUTPUTS[k]
        if name == "demod":
            return True
        if name == "audio":
            return bool(self.flags & (SDR_RX_AUDIO | SDR_RX_STEREO))
        if k <= RX_OUTPUTS.index("right"):
            return bool(self.flags & SDR_RX_STEREO)
        return bool(self.flags & SDR_RX_RDS)

    def _call(self, fn, iq, fetch):
        es = np.uint8 if self.u8 else np.float32
        iq = np.ascontiguousarray(iq, dtype=es)
        if iq.size != self.S * 2 * self.B:
            raise ValueError(f"expected {self.S} x {2 * self.B} interleaved values, got {iq.shape}")
        key = tuple(fetch) if fetch is not None else None
        plan = self._plans.get(key)
        if plan is None:                      # output names -> (which[], lengths, offsets), built once
            names = list(fetch) if fetch is not None else \
                [n for n in ("audio", "left", "right", "rrc_i", "rrc_q") if n in self.outputs]
            which = (ctypes.c_int * len(names))(*[RX_OUTPUTS.index(n) for n in names])
            lengths = [self._length(n) for n in names]
            offs = [self.S * sum(lengths[:i]) for i in range(len(names))]
            plan = self._plans[key] = (names, which, lengths, offs, self.S * sum(lengths),
                                       ctypes.c_void_p * len(names))
        names, which, lengths, offs, total, ptr_array = plan
        # one allocation per call, the outputs (S, n) views of it
        buf = np.empty(max(total, 1), dtype=np.float32)
        base = _addr(buf)
        ptrs = ptr_array(*[base + 4 * o for o in offs])
        outs = {n: buf[o:o + self.S * m].reshape(self.S, m) for n, o, m in zip(names, offs, lengths)}
        check(getattr(self.lib, fn)(self.handle, _addr(iq), self.B, len(names), which, ptrs, None), fn)
        return outs

    def process(self, iq, fetch=None):
        """One block of every stream; returns {name: (nstreams, n) float32} for `fetch`
        (default: the configuration's final outputs).  One C call: IQ up, the chain, the
        outputs down, one wait (sdr_rx_run)."""
        if self._pending:                     # submitted blocks are delivered (and dropped) first
            self.flush()
        return self._call("sdr_rx_run", iq, fetch)

    def submit(self, iq, fetch=None):
        """process() without waiting (sdr_rx_submit): launches this block and returns the
        outputs of the block submitted `depth` calls earlier (None while the pipeline fills:
        depth 1 = the PREVIOUS block), so the host prepares the next block while these run.
        flush() returns the rest."""
        self._pending.append(self._call("sdr_rx_submit", iq, fetch))
        return self._pending.popleft() if len(self._pending) > self.depth else None

    def flush(self):
        """Wait for every submitted block; returns the list of the blocks' outputs not yet
        returned by submit(), oldest first (empty when none is in flight), at any depth."""
        check(self.lib.sdr_rx_flush(self.handle), "sdr_rx_flush")
        rest = list(self._pending)
        self._pending.clear()
        return rest

    def _length(self, name):
        if name not in self._lengths:
            self._lengths[name] = self.output_ptr(name)[2]
        return self._lengths[name]

    def set_keep(self, names):
        """Outputs process_dev materialises (sdr_rx_set_keep; default: all).  Leaving out the
        NCO rows ("nco", "nco_i", "nco_q") and the RDS LPF rows ("lpf_i", "lpf_q") -- which the
        chain itself does not need -- keeps them out of HBM: the mixers form the NCO from the PLL
        phases and the RDS LPF runs inside the composite resampler (the same values either way).
        process() / submit() materialise what they are asked for."""
        mask = 0
        for n in names:
            mask |= 1 << RX_OUTPUTS.index(n)
        check(self.lib.sdr_rx_set_keep(self.handle, mask), "sdr_rx_set_keep")

    def process_dev(self, iq_ptr: int, iq_stride: int):
        """One block from device memory (async on the context stream); outputs stay on the
        GPU (output_ptr)."""
        check(self.lib.sdr_rx_process_dev(self.handle, iq_ptr, int(iq_stride)), "sdr_rx_process_dev")

    def output_ptr(self, name: str):
        """(device pointer, row stride in floats, samples per row) of output `name`."""
        p, st, n = ctypes.c_void_p(), ctypes.c_int64(), ctypes.c_int64()
        check(self.lib.sdr_rx_output(self.handle, RX_OUTPUTS.index(name), ctypes.byref(p), ctypes.byref(st),
                                     ctypes.byref(n)), "sdr_rx_output")
        return p.value, st.value, n.value

    def output(self, name: str) -> np.ndarray:
        _, _, n = self.output_ptr(name)
        out = np.empty((self.S, n), dtype=np.float32)
        check(self.lib.sdr_rx_fetch(self.handle, RX_OUTPUTS.index(name), out.ctypes.data_as(_lib._fp), n),
              "sdr_rx_fetch")
        return out

    def state(self):
        """Carried states: (demod prev_phase [S], stereo PLL [S, 6], RDS PLL [S, 6])."""
        ph = np.empty(self.S)
        ps, pr = np.empty((self.S, 6)), np.empty((self.S, 6))
        check(self.lib.sdr_rx_state(self.handle, f64p(ph), f64p(ps), f64p(pr)), "sdr_rx_state")
        return ph, ps, pr

    def pll_stats(self, reset: bool = False) -> dict:
        """How the PLL recurrences were solved (sdr_rx_pll_stats: the context's counters, after
        every block in flight): counts by solver; see _lib.PLL_STATS."""
        return _lib.decode_pll_stats(lambda a: self.lib.sdr_rx_pll_stats(self.handle, a.ctypes.data,
                                                                         int(bool(reset))))

    def reset(self):
        check(self.lib.sdr_rx_reset(self.handle), "sdr_rx_reset")
        self._pending.clear()

    def set_timing(self, on: bool = True):
        """Record HIP events between the receiver's launches (stage_ms)."""
        check(self.lib.sdr_rx_set_timing(self.handle, int(bool(on))), "sdr_rx_set_timing")

    def stage_ms(self) -> dict:
        """GPU time per stage of the last block (set_timing(True) first): _lib.RX_STAGES."""
        ms = np.zeros(len(_lib.RX_STAGES), dtype=np.float32)
        check(self.lib.sdr_rx_stage_ms(self.handle, ms.ctypes.data_as(_lib._fp)), "sdr_rx_stage_ms")
        return dict(zip(_lib.RX_STAGES, (float(v) for v in ms)))

    def close(self):
        if getattr(self, "handle", None):
            self.lib.sdr_rx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class MonoBlockProcessor:
    """FE (RF LPF + decimate + atan2 demod) and mono audio LPF + decimate per block.

    block_complex: complex samples per block (model/fmMonoBlock.py:53 uses 51 200)."""

    _mode = dict(mono=True)

    def __init__(self, block_complex: int, rf_coeff=None, audio_coeff=None, rf_decim: int = 10,
                 audio_decim: int = 5, iq_dtype=np.float32, ctx=None, **kw):
        self.B = int(block_complex)
        self.rx = Receiver(1, self.B, iq_dtype=iq_dtype, rf_coeff=rf_coeff, audio_coeff=audio_coeff,
                           rf_decim=rf_decim, audio_decim=audio_decim, ctx=ctx, **self._mode, **kw)
        self.ctx = self.rx.ctx
        self.M, self.A = self.rx.M, self.rx.A

    def _run(self, iq_block, names):
        iq = np.asarray(iq_block)
        if iq.shape != (2 * self.B,):
            raise ValueError(f"expected {2 * self.B} interleaved values, got {iq.shape}")
        o = self.rx.process(iq, fetch=names)
        return {k: v[0].astype(np.float64) for k, v in o.items()}

    def process(self, iq_block, return_demod: bool = False):
        """audio_block (float64) for one block [+ fm_demod]."""
        o = self._run(iq_block, ["audio", "demod"] if return_demod else ["audio"])
        return (o["audio"], o["demod"]) if return_demod else o["audio"]

    @property
    def phase(self) -> float:
        """The carried demod phase (model/fmSupportLib.py:40-44)."""
        return float(self.rx.state()[0][0])


class StereoBlockProcessor(MonoBlockProcessor):
    """Mono + stereo (model/fmMonoBlock.py:113-173, intended combiner L=(a+s)/2, R=(a-s)/2)."""

    _mode = dict(mono=True, stereo=True)

    def __init__(self, block_complex: int, rf_coeff=None, audio_coeff=None, stereo_taps: int = 151, **kw):
        super().__init__(block_complex, rf_coeff, audio_coeff, stereo_taps=stereo_taps, **kw)

    def process(self, iq_block, return_intermediates: bool = False):
        names = ["audio", "stereo", "left", "right"]
        if return_intermediates:
            names += ["demod", "bpf_recovery", "nco", "bpf_extraction"]
        return self._run(iq_block, names)


class RdsBlockProcessor(MonoBlockProcessor):
    """RDS signal path of model/fmRDSblock.py:156-204, from the demod stream to the RRC
    output (I and Q).  The bit-level link layer after :204 is RdsLinkLayer."""

    _mode = dict(mono=False, rds=True)

    def __init__(self, block_complex: int = 153600, rf_coeff=None, taps: int = 151, iq_dtype=np.uint8, **kw):
        super().__init__(block_complex, rf_coeff, None, iq_dtype=iq_dtype, rds_taps=taps, **kw)
        self.R = self.rx.R

    def process(self, iq_block, return_intermediates: bool = False):
        names = ["rrc_i", "rrc_q"]
        if return_intermediates:
            names += ["demod", "extract", "pre_pll", "nco_i", "nco_q", "lpf_i", "lpf_q", "resample_i",
                      "resample_q"]
        return self._run(iq_block, names)


class RdsLinkLayer:
    """RDS link layer of model/fmRDSblock.py:207-346 on the host (libsdr C++, no GPU):
    clock and data recovery, Manchester and differential decoding, syndrome frame sync.

    process(rrc_i) takes one block of the in-phase RRC output (RdsBlockProcessor's
    'rrc_i') and returns dict(events=[(type, position, accepted)], symbols, bits, diff):
    type 0..3 = syndrome A..D, accepted = the reference's "Syndrome X at position N"
    prints (1) or its "False positive" prints (0); the state carries across calls."""

    TYPES = "ABCD"
    RESYNC = 4

    def __init__(self, resync_after: int = 0):
        """resync_after > 0: the C++ frame_thread's rule (src/fm_radio.cpp:697-704; it uses
        10) -- after that many false positives in a row the frame position is forgotten and a
        (RESYNC, position, 0) event is reported.  0: the Python model's behaviour."""
        import ctypes
        self._c = ctypes
        self.lib = _lib.load_library()
        h = ctypes.c_void_p()
        check(self.lib.sdr_rds_link_create(ctypes.byref(h)), "sdr_rds_link_create")
        self.handle = h
        if resync_after:
            check(self.lib.sdr_rds_link_set_resync(h, int(resync_after)), "sdr_rds_link_set_resync")

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
