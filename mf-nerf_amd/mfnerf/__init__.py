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

# HIP graph replays through the runtime's per-node launch path instead of its captured-packet path:
# ~5 -> ~1 us per graph launch on a probe (tools/probe_graph_gap.py), 0.5666 -> 0.5632 ms per
# training step A/B (profiles/r03_v6_ab_graph_packet_capture.txt).  Read when the HIP runtime
# initialises, so it applies when this package is imported first; an explicit setting wins.
os.environ.setdefault("DEBUG_CLR_GRAPH_PACKET_CAPTURE", "0")

from . import _lib  # noqa: E402

__all__ = ["vren", "custom_functions", "rendering", "networks", "losses", "tcnn", "field", "grid", "engine"]


def lib_path():
    return _lib.LIB_PATH
