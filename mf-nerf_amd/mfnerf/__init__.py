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
import os

# HIP graph replays through the runtime's per-node launch path instead of its captured-packet path
# (DEBUG_CLR_GRAPH_PACKET_CAPTURE=0): ~5 -> ~1 us per graph launch on a probe
# (tools/probe_graph_gap.py), 0.5666 -> 0.5632 ms per training step A/B
# (profiles/r03_v6_ab_graph_packet_capture.txt).  The variable is process-wide (it changes how every
# HIP graph of the host application launches) and is read once when the HIP runtime initialises, so
# the package only sets it on request: MFNERF_GRAPH_NODE_LAUNCH=1 before importing it (bench.py and
# tools/train_30k.py set the variable themselves, before torch).
if os.environ.get("MFNERF_GRAPH_NODE_LAUNCH", "0") == "1":
    import sys as _sys
    _torch = _sys.modules.get("torch")
    if _torch is not None and _torch.cuda.is_initialized():
        import warnings as _warnings
        _warnings.warn("MFNERF_GRAPH_NODE_LAUNCH=1 has no effect: the HIP runtime was initialised before "
                       "mfnerf was imported (set DEBUG_CLR_GRAPH_PACKET_CAPTURE=0 before the first HIP call)")
    os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

from . import _lib  # noqa: E402

__all__ = ["vren", "custom_functions", "rendering", "networks", "losses", "tcnn", "field", "grid", "engine"]


def lib_path():
    return _lib.LIB_PATH
