"""MI355X-native FM-SDR hot path (gfx950 HIP kernels behind a ctypes C-ABI).

Import with ``importlib.import_module("real-time-software-defined-radio_amd")`` (the
directory name is not an identifier) or ``import rtsdr`` from the repo root.

Drop-in per-block functions with the reference's names and signatures
(model/fmSupportLib.py, model/fmPll.py, model/fmRRC.py, scipy.signal.lfilter):

    lfilter, fmDemodArctan, fmPll, my_convoloution, impulseResponseRootRaisedCosine,
    my_filterImpulseResponse

fused hot-path forms: lfilter_decim, rf_frontend_block, mono_block, resample,
fm_mono_streams;
device-resident block pipelines: MonoBlockProcessor, StereoBlockProcessor,
RdsBlockProcessor.  See DESIGN.md and INTEGRATION.md.
"""
from . import design, synth  # noqa: F401
from ._lib import (SDR_IQ_F32, SDR_IQ_U8, SDR_PRE_MIX, SDR_PRE_NONE, SDR_PRE_SQUARE, Context,  # noqa: F401
                   DeviceBuffer, SdrError, SdrUnavailable, Timer, device_count, device_info, get_context,
                   load_library)
from .blocks import MonoBlockProcessor, RdsBlockProcessor, RdsLinkLayer, Receiver, StereoBlockProcessor  # noqa: F401
from .design import impulseResponseRootRaisedCosine, my_filterImpulseResponse  # noqa: F401
from .dsp import (DFT, MonoState, estimatePSD, fm_mono_range, fm_mono_streams, split_halo, fmDemodArctan, fmPll, lfilter, lfilter_decim,  # noqa: F401
                  mono_block, my_convoloution, resample, rf_frontend_block)

__version__ = "0.1.0"
