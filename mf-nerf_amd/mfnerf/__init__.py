"""mfnerf: MI355X-native (gfx950 HIP) kernels behind MF-NeRF's volumetric-rendering training step.

Drop-in layers (same names and behaviour as the reference):
  mfnerf.vren               <- models/csrc `vren` pybind module
  mfnerf.custom_functions   <- models/custom_functions.py
  mfnerf.rendering          <- models/rendering.py
  mfnerf.networks.NGP       <- models/networks.py (tcnn modules replaced by fused HIP kernels)
  mfnerf.losses             <- losses.py
  mfnerf.tcnn               <- the tinycudann subset MF-NeRF configures
Fast path: mfnerf.engine.TrainStep (device-resident sample counts, no host syncs).
All GPU work goes through libmfnerf_hip.so (include/mfnerf.h); there is no CPU fallback.
"""
from . import _lib

__all__ = ["vren", "custom_functions", "rendering", "networks", "losses", "tcnn", "field", "grid", "engine"]


def lib_path():
    return _lib.LIB_PATH
