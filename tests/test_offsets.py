"""Input realism for the PLLs: a transmitter pilot off its nominal 19 kHz (the FM standard
allows +-2 Hz; the stereo subcarrier and the RDS 57 kHz subcarrier move with it, so the RDS
PLL's 114 kHz carrier moves 6x) and an RTL-SDR sample clock 50 ppm fast (src/iofunc.cpp:61-69
takes whatever the dongle delivers: every tone seen 50 ppm low -- the pilot -0.95 Hz, the RDS
carrier -5.7 Hz).  Synthetic composite resampled accordingly (synth.fm_iq pilot_offset_hz,
clock_ppm).

One u8 stream, 3 blocks of 153 600 (src/fm_radio.cpp:23), mono + stereo + RDS through the
block receiver, against the oracle's block loops (model/fmMonoBlock.py:80-173,
model/fmRDSblock.py:127-204); and the parallel solve's hit rate on the blocks after the first
(the acquisition block), from the solver counters.  The table is printed (pytest -s) and
recorded in profiles/r03/offsets.txt."""
import numpy as np
import pytest

from conftest import long_blocks, maxabs, rms
from test_receiver import AUDIO_MAX, AUDIO_RMS, NCO_MAX, RDS_TOL

pytestmark = pytest.mark.gpu

B5 = 153_600
NB = 3
CASES = [(0.0, 0.0), (2.0, 0.0), (-2.0, 0.0), (5.0, 0.0), (-5.0, 0.0), (0.0, 50.0), (0.0, -50.0)]


@pytest.mark.parametrize("offset,ppm", CASES)
def test_offsets_match_oracle(sdr, gpu_ctx, oracle, offset, ppm):
    iq = sdr.synth.fm_iq(NB * B5 + 1, seed=90, dtype=np.uint8, pilot_offset_hz=offset, clock_ppm=ppm)
    rx = sdr.Receiver(1, B5, stereo=True, rds=True, iq_dtype=np.uint8)
    names = ["audio", "stereo", "left", "right", "nco"] + list(RDS_TOL)
    got = []
    for k in range(NB):
        got.append(rx.process(iq[2 * k * B5:2 * (k + 1) * B5], fetch=names))
        if k == 0:
            rx.pll_stats(reset=True)          # count the blocks after the acquisition block
    st = rx.pll_stats()
    f = (iq.astype(np.float64) - 128.0) / 128.0
    mono = oracle.mono_stereo_blocks(f, B5, rf_taps=151, audio_taps=151, nblocks=NB)
    rds = oracle.rds_blocks(iq, 2 * B5, taps=151, nblocks=NB)
    nco_err = 0.0
    for k in range(NB):
        g = got[k]
        for key in ("audio", "stereo", "left", "right"):
            assert rms(g[key][0], mono[k][key]) < AUDIO_RMS, (key, k)
            assert maxabs(g[key][0], mono[k][key]) < AUDIO_MAX, (key, k)
        nco_err = max(nco_err, maxabs(g["nco"][0], mono[k]["nco"]))
        assert maxabs(g["nco"][0], mono[k]["nco"]) < NCO_MAX, k
        for key, (tmax, trms) in RDS_TOL.items():
            ref = rds[k][key]
            scale = max(float(np.max(np.abs(ref))), 1e-3)
            em, er = maxabs(g[key][0], ref) / scale, rms(g[key][0], ref) / scale
            assert em < tmax and er < trms, (key, k, em, er)
    hits = st["spec_r0"] + st["spec_r1"] + st["spec_r2"]
    print(f"pilot offset {offset:+.1f} Hz, clock {ppm:+.0f} ppm: parallel solve {hits}/{st['recurrences']} "
          f"recurrences of blocks 1-{NB - 1} (round 0: {st['spec_r0']}, sequential: {st['sequential']}); "
          f"stereo NCO max err {nco_err:.1e}")
    assert st["recurrences"] == 2 * (NB - 1) * long_blocks(B5 // 10)
    # the FM standard's +-2 Hz and a 50 ppm crystal are solved in parallel on every locked block
    if abs(offset) <= 2.0:
        assert hits == st["recurrences"], st
