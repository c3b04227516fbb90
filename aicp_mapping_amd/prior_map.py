"""Device-resident prior map of aicp_core's localization mode.

App keeps ``prior_map_`` (an AlignedCloud) and, in localization mode:
- crops it around each reading's prior pose to make the reference (``setReference``,
  app.cpp:41-51, ``getPointsInOrientedBox`` filteringUtils.cpp:619-637);
- appends the aligned reading every ``reference_update_frequency`` clouds when
  ``merge_aligned_clouds_to_map`` (app.cpp:469-483: ``*merged_map = *prior_map + *output`` with
  ``output = transformPointCloud(read_prefiltered, correction)``);
- pre-filters the whole map every 30 clouds (app.cpp:485-493).

``PriorMap`` holds the map in HBM (aicp_hip_map_*) so none of these steps re-uploads it.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib as L


class PriorMap:
    def __init__(self, ctx: "L.Context", points):
        pts = L.as_points(points)
        h = C.c_void_p()
        ctx.check(L.lib.aicp_hip_map_create(ctx.h, L._fptr(pts), pts.shape[0], pts.shape[1] * 4, C.byref(h)))
        self.ctx = ctx
        self.h = h

    def free(self):
        if getattr(self, "h", None):
            L.lib.aicp_hip_map_free(self.ctx.h, self.h)
            self.h = None

    def __del__(self):
        self.free()

    def __len__(self):
        n = C.c_size_t()
        L.lib.aicp_hip_map_size(self.h, C.byref(n))
        return n.value

    def getCloud(self) -> np.ndarray:
        """The map's points (AlignedCloud::getCloud), (N, 3) float32."""
        n = len(self)
        out = np.zeros((max(n, 1), 3), np.float32)
        m = C.c_size_t()
        self.ctx.check(L.lib.aicp_hip_map_download(self.ctx.h, self.h, L._fptr(out), n, C.byref(m)))
        return out[:m.value].copy()

    def crop(self, mn: float, mx: float, origin) -> np.ndarray:
        """getPointsInOrientedBox(map, mn, mx, origin) on device; origin a 4x4 pose (row-major)."""
        o = np.ascontiguousarray(np.asarray(origin, np.float32).reshape(4, 4).T.reshape(16))
        n = len(self)
        out = np.zeros((max(n, 1), 3), np.float32)
        m = C.c_size_t()
        self.ctx.check(L.lib.aicp_hip_map_crop(self.ctx.h, self.h, float(mn), float(mx), L._fptr(o), L._fptr(out),
                                               n, C.byref(m)))
        return out[:m.value].copy()

    def register_batch(self, readings, poses, mn: float = -15.0, mx: float = 15.0, cfg=None, flags: int = 0):
        """Localization-only registration of a batch (aicp_hip_map_register_batch): reading i
        against this map cropped on the device around poses[i] (4x4 row-major prior pose), overlap
        fixed at 50 % (app.cpp:41-51,123-127). readings: list of (N, 3|4|8|12) float32 rows.
        Returns (T[n, 4, 4] row-major, list of stats dicts, rc)."""
        cfg = cfg or L.default_config()
        n = len(readings)
        arr = (L.Cloud * n)()
        keep = []
        for i, r in enumerate(readings):
            P = np.asarray(poses[i], np.float64).reshape(4, 4)
            c, k = L.make_cloud(r, P[:3, 3])
            arr[i] = c
            keep.append(k)
        pz = np.ascontiguousarray(np.stack([np.asarray(p, np.float32).reshape(4, 4).T.reshape(16) for p in poses]))
        outT = np.zeros((n, 16), np.float32)
        st = (L.IcpStats * n)()
        rc = L.lib.aicp_hip_map_register_batch(self.ctx.h, C.byref(cfg), self.h, float(mn), float(mx), arr, L._fptr(pz),
                                               n, int(flags), L._fptr(outT), st)
        if rc != L.AICP_OK:
            self.ctx.check(rc)
        return outT.reshape(-1, 4, 4).transpose(0, 2, 1).copy(), [x.as_dict() for x in st], rc

    def merge(self, points, correction) -> None:
        """*map = *map + transformPointCloud(points, correction); correction a 4x4 (row-major)."""
        pts = L.as_points(points)
        t = np.ascontiguousarray(np.asarray(correction, np.float32).reshape(4, 4).T.reshape(16))
        self.ctx.check(L.lib.aicp_hip_map_merge(self.ctx.h, self.h, L._fptr(pts), pts.shape[0], pts.shape[1] * 4,
                                                L._fptr(t)))

    def prefilter(self, params=None) -> None:
        """map = regionGrowingUniformPlaneSegmentationFilter(map) on device."""
        prm = params or L.default_prefilter()
        self.ctx.check(L.lib.aicp_hip_map_prefilter(self.ctx.h, self.h, C.byref(prm)))


def localization_update(prior_map: PriorMap, read_prefiltered, correction, n_clouds: int,
                        reference_update_frequency: int = 5, merge_aligned_clouds_to_map: bool = True,
                        is_reference: bool = False) -> None:
    """App's map maintenance after an accepted alignment in localization mode (app.cpp:469-493);
    n_clouds = aligned_clouds_graph_->getNbClouds() after adding the reading."""
    if not is_reference and (n_clouds - 1) % reference_update_frequency == 0 and merge_aligned_clouds_to_map:
        prior_map.merge(read_prefiltered, correction)
    if merge_aligned_clouds_to_map and (n_clouds - 1) % 30 == 0:
        prior_map.prefilter()
