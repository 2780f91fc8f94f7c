"""`import rtsdr` == the package in real-time-software-defined-radio_amd/ (whose
directory name is not a Python identifier)."""
import importlib
import os
import sys

_ROOT = os.path.dirname(os.path.abspath(__file__))
if _ROOT not in sys.path:
    sys.path.insert(0, _ROOT)
sys.modules[__name__] = importlib.import_module("real-time-software-defined-radio_amd")
