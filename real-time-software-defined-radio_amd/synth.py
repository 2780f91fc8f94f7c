"""Seeded synthetic FM-broadcast IQ (the reference ships no captures: data/simple_readme.txt).

Composite baseband: mono L+R, 19 kHz pilot, L-R on a 38 kHz
subcarrier, and +-1 RDS symbols at 2375 Bd on 57 kHz; frequency-modulated with
75 kHz deviation at 2.4 MS/s; complex AWGN at 30 dB SNR.  Output is interleaved
[I0, Q0, I1, Q1, ...] float32 (model/fmMonoBlock.py:39) or uint8
(model/fmRDSblock.py:58, as rtl_sdr produces).
"""
from __future__ import annotations

import numpy as np

FS = 2.4e6


# RDS block coding (IEC 62106): 26-bit blocks = 16 information bits + 10-bit checkword,
# checkword = (m(x) x^10 mod g(x)) XOR offset word; g(x) = x^10+x^8+x^7+x^5+x^4+x^3+1.
RDS_POLY = 0x5B9
RDS_OFFSETS = {"A": 0x0FC, "B": 0x198, "C": 0x168, "D": 0x1B4}


def rds_block_bits(info: int, offset: str) -> list:
    """26 bits (MSB first) of one RDS block."""
    reg = (info & 0xFFFF) << 10
    for b in range(25, 9, -1):
        if reg & (1 << b):
            reg ^= RDS_POLY << (b - 10)
    word = ((info & 0xFFFF) << 10) | ((reg & 0x3FF) ^ RDS_OFFSETS[offset])
    return [(word >> (25 - k)) & 1 for k in range(26)]


def rds_symbols(nbits: int, seed: int = 0) -> np.ndarray:
    """+-1 biphase symbols (2 per bit, 2375 symbols/s) of a stream of RDS groups (A B C D
    blocks, random information words): differential encoding e_t = e_(t-1) xor d_t, then
    Manchester e=1 -> (+1, -1), e=0 -> (-1, +1) -- the inverse of the decoder in
    model/fmRDSblock.py:250-292."""
    rng = np.random.default_rng(seed)
    bits = []
    while len(bits) < nbits:
        for off in "ABCD":
            bits += rds_block_bits(int(rng.integers(0, 1 << 16)), off)
    e, sym = 0, np.empty(2 * nbits)
    for t in range(nbits):
        e ^= bits[t]
        sym[2 * t], sym[2 * t + 1] = (1.0, -1.0) if e else (-1.0, 1.0)
    return sym


def fm_iq(n_complex: int, seed: int = 0, fs: float = FS, snr_db: float = 30.0, chunk: int = 1 << 22,
          dtype=np.float32, rds_groups: bool = False, rds_phase: float = 0.0, pilot_offset_hz: float = 0.0,
          clock_ppm: float = 0.0) -> np.ndarray:
    """Interleaved float32 IQ of `n_complex` samples (generated in chunks to bound memory).
    rds_groups: the 57 kHz subcarrier carries coded RDS groups (rds_symbols) at carrier
    phase `rds_phase` instead of random symbols.
    pilot_offset_hz: the transmitter's pilot is 19 kHz + offset, and the 38 / 57 kHz
    subcarriers derived from it move with it (x2, x3; the RDS PLL's 114 kHz carrier x6).
    clock_ppm: the receiver's sample clock runs fast by this many ppm (an RTL-SDR crystal's
    error, src/iofunc.cpp:61-69 reads whatever it delivers): sample k is taken at transmitter
    time k / (fs (1 + ppm 1e-6)), so every tone, the RDS symbol rate and the FM phase
    integral are seen slightly slow -- the composite resampled."""
    rng = np.random.default_rng(seed)
    out = np.empty(2 * n_complex, dtype=np.float32)
    fs_tx = fs * (1.0 + clock_ppm * 1e-6)       # receiver samples per transmitter second
    fp = 19e3 + pilot_offset_hz
    sym_len = fs_tx / 2375.0
    nsym = int(np.ceil(n_complex / sym_len)) + 2
    symbols = rng.choice(np.array([-1.0, 1.0]), size=nsym)
    if rds_groups:
        symbols = rds_symbols((nsym + 1) // 2, seed)[:nsym]
    noise_rng = np.random.default_rng(seed + 1_000_003)
    amp = 0.5
    sigma = amp / np.sqrt(2.0) * 10 ** (-snr_db / 20.0)
    phase0 = 0.0
    for start in range(0, n_complex, chunk):
        n = min(chunk, n_complex - start)
        t = (start + np.arange(n, dtype=np.float64)) / fs_tx
        left = np.sin(2 * np.pi * 1e3 * t)
        right = 0.8 * np.sin(2 * np.pi * 2.5e3 * t)
        rds = symbols[((start + np.arange(n)) / sym_len).astype(np.int64)]
        mpx = (0.45 * (left + right) / 2 + 0.1 * np.cos(2 * np.pi * fp * t)
               + 0.45 * (left - right) / 2 * np.cos(2 * np.pi * (2 * fp) * t)
               + 0.05 * rds * np.cos(2 * np.pi * (3 * fp) * t + rds_phase))
        phi = phase0 + 2 * np.pi * 75e3 * np.cumsum(mpx) / fs_tx
        phase0 = float(phi[-1])
        noise = noise_rng.standard_normal((n, 2)) * sigma
        out[2 * start:2 * (start + n):2] = (amp * np.cos(phi) + noise[:, 0]).astype(np.float32)
        out[2 * start + 1:2 * (start + n):2] = (amp * np.sin(phi) + noise[:, 1]).astype(np.float32)
    if np.dtype(dtype) == np.uint8:
        return to_u8(out)
    return out


def to_u8(iq: np.ndarray) -> np.ndarray:
    """round(127 * x / max|x| + 128), the rtl_sdr-style byte stream."""
    peak = float(np.max(np.abs(iq))) or 1.0
    return np.clip(np.rint(127.0 * iq / peak + 128.0), 0, 255).astype(np.uint8)
