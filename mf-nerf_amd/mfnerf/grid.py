"""Host-side level table of the multiresolution grid encoding.

Mirrors tiny-cuda-nn's GridEncodingTemplated constructor sizing (the encoding configured at
models/networks.py:36-49): per level l, scale_l = exp2f(l * log2f(b)) * N_min - 1 evaluated in
fp32 exactly as tcnn does (b is read from the JSON config as a float), res_l = ceil(scale_l)+1,
params_l = min(next_multiple(res_l^3, 8), 2^log2_T).  At the default Lego config this gives
11,445,040 table params (levels 5/10/15 land on res 65/257/1025 because log2f(float(b)) rounds
up; SURVEY.md's 11,420,064 assumed log2 b = 0.4 exactly) -- see DESIGN.md.

MixedFeature ("MixedFeatureGrid", opt.py:71-73): the levels that own a dense table keep it; the
hashed levels share `n_tables` tables holding 2^log2_T entries in total, level l using table
(l - first_hashed) % n_tables, and index a point through its coordinates on the canonical
(finest) grid, so coincident points of different levels share features (this repo's reading of
arXiv 2304.12587; the fork's code is absent, parity unpinned).
"""
import ctypes
import ctypes.util
import math

from ._lib import MAX_LEVELS, GridDesc

_libm = ctypes.CDLL(ctypes.util.find_library("m") or "libm.so.6")
_libm.log2f.restype = ctypes.c_float
_libm.log2f.argtypes = [ctypes.c_float]
_libm.exp2f.restype = ctypes.c_float
_libm.exp2f.argtypes = [ctypes.c_float]


def _f32(x):
    return ctypes.c_float(x).value


class GridLayout:
    def __init__(self, n_levels=16, n_features=2, log2_T=19, base_res=16, per_level_scale=2.0, grid="Hash",
                 n_tables=1):
        if n_levels > MAX_LEVELS:
            raise ValueError(f"n_levels <= {MAX_LEVELS}")
        self.L, self.F, self.log2_T, self.N_min = int(n_levels), int(n_features), int(log2_T), int(base_res)
        self.b = float(per_level_scale)
        self.grid = grid
        self.mixed = grid == "MixedFeature"
        self.n_tables = max(1, int(n_tables))
        T = 1 << self.log2_T
        log2b = _libm.log2f(_f32(self.b))
        self.scales, self.res = [], []
        for l in range(self.L):
            e = _libm.exp2f(_f32(_f32(float(l)) * log2b))
            s = _f32(_f32(e * _f32(float(self.N_min))) - 1.0)
            self.scales.append(s)
            self.res.append(int(math.ceil(s)) + 1)
        hashed = [l for l in range(self.L) if self.res[l] ** 3 > T]
        self.kind, self.offsets, self.sizes = [], [], []
        off = 0
        for l in range(self.L):
            if self.mixed and l in hashed:
                self.kind.append(1)
                self.offsets.append(-1)
                self.sizes.append(0)
                continue
            p = min(self.res[l] ** 3, 0x7FFFFFFF)
            p = min((p + 7) // 8 * 8, T)
            self.kind.append(0)
            self.offsets.append(off)
            self.sizes.append(p)
            off += p
        if self.mixed and hashed:
            shared = max(8, (T // self.n_tables) // 8 * 8)
            for i, l in enumerate(hashed):
                self.offsets[l] = off + (i % self.n_tables) * shared
                self.sizes[l] = shared
            off += shared * self.n_tables
        self.n_entries = off
        self.n_params = off * self.F
        self.canon_res = self.res[-1]

    def desc(self):
        d = GridDesc()
        d.n_levels, d.n_features, d.canon_res = self.L, self.F, self.canon_res
        for l in range(self.L):
            d.scale[l] = self.scales[l]
            d.res[l] = self.res[l]
            d.offset[l] = self.offsets[l]
            d.size[l] = self.sizes[l]
            d.table_kind[l] = self.kind[l]
        return d

    @staticmethod
    def from_config(cfg):
        return GridLayout(cfg["n_levels"], cfg["n_features_per_level"], cfg["log2_hashmap_size"],
                          cfg["base_resolution"], cfg["per_level_scale"], cfg.get("type", "Hash"),
                          cfg.get("n_tables", 1))
