set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_live.py tests/test_rds_link.py -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_live.log 2>&1
python3 -c "
import sys; sys.path.insert(0,'.'); import rtsdr, numpy as np
rtsdr.synth.fm_iq(200*153600, seed=3, dtype=np.uint8).tofile('/tmp/live_u8.raw')"
S=$(date +%s.%N); timeout -k 10 120 real-time-software-defined-radio_amd/fm_radio_gpu < /tmp/live_u8.raw > /tmp/live.pcm 2> gpurun_out/live_err.log; E=$(date +%s.%N)
python3 -c "print('stereo: 200 blocks x 153600 complex in %.3f s -> %.1f MS/s' % ($E-$S, 200*153600/($E-$S)/1e6))" > gpurun_out/live_time.log
S=$(date +%s.%N); timeout -k 10 120 real-time-software-defined-radio_amd/fm_radio_gpu --mono < /tmp/live_u8.raw > /tmp/live.pcm 2>> gpurun_out/live_err.log; E=$(date +%s.%N)
python3 -c "print('mono: 200 blocks x 153600 complex in %.3f s -> %.1f MS/s' % ($E-$S, 200*153600/($E-$S)/1e6))" >> gpurun_out/live_time.log
