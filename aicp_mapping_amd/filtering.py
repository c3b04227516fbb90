"""Host mirror of aicp_core's pre-filter (aicp_core/include/aicp_utils/filteringUtils.hpp:29-34,
aicp_core/src/utils/filteringUtils.cpp:5-103), SURVEY.md §8(f) rank 2.

Both overloads run on the device through aicp_hip_prefilter (kernels_prefilter.hip):
VoxelGrid 0.08 -> NormalEstimation k = 30 -> RegionGrowing (15 neighbours, 3 deg smoothness,
curvature 1.0, clusters of 50..1e6 points). There is no CPU fallback.
"""
from __future__ import annotations

import numpy as np

from . import _lib

_CTX = None


def _ctx(ctx):
    global _CTX
    if ctx is not None:
        return ctx
    if _CTX is None:
        _CTX = _lib.Context(0)
    return _CTX


def _cluster_rgb(c: int) -> float:
    """Colour of cluster c as the reference stores it: ``points[idx].rgb = rgb`` with an int32
    ``rgb = (r << 16) | (g << 8) | b`` (filteringUtils.cpp:92-100) is a numeric int -> float
    conversion of the float field, not a bit-packed colour, and so it is here. The reference draws
    r, g, b at random (srand(time(NULL)), :89); a fixed hash of the cluster index here, so runs
    are repeatable."""
    h = (c * 2654435761 + 12345) & 0xFFFFFFFF
    rgb = ((h >> 8) & 0xFF) << 16 | ((h >> 16) & 0xFF) << 8 | ((h >> 24) & 0xFF)
    return float(np.float32(rgb))


def regionGrowingUniformPlaneSegmentationFilter(cloud_in, *args, ctx=None, params=None):
    """filteringUtils.cpp overloads, as in the reference:

    - ``regionGrowingUniformPlaneSegmentationFilter(cloud_in[, cloud_out])`` (:5-45): returns the
      points of the kept plane clusters, clusters concatenated in creation order, each in
      sampled-cloud order, appended to ``cloud_out`` when given (``*cloud_out = *cloud_out +
      cloud_cluster``).
    - ``regionGrowingUniformPlaneSegmentationFilter(cloud_in, view_point, clusters)`` (:51-103,
      view_point a 4x4 pose, clusters a list to fill like ``std::vector<pcl::PointIndices>&``):
      returns the sampled cloud as (V, 12) PointXYZRGBNormal rows {x, y, z, 1, nx, ny, nz, 0,
      rgb, curvature, 0, 0}; normals face view_point.translation(); each kept cluster's points
      carry one colour (rgb = float(int32 colour), the reference's numeric conversion).

    cloud_in: (N, 3|4|8|12) float32 rows. ctx: an aicp Context (default: one on device 0)."""
    if len(args) > 2:
        raise TypeError("expected (cloud_in[, cloud_out]) or (cloud_in, view_point, clusters)")
    c = _ctx(ctx)
    if len(args) == 2:
        view_point, clusters = args
        T = np.asarray(view_point, np.float64).reshape(4, 4)
        # a copy: the caller's params keep their own viewpoint (the first overload's is (0,0,0))
        prm = _lib.PrefilterParams.from_buffer_copy(params) if params is not None else _lib.default_prefilter()
        for i in range(3):
            prm.viewpoint[i] = float(np.float32(T[i, 3]))
        r = c.prefilter(cloud_in, prm, details=True)
        s, lab = r["sampled"], r["labels"]
        out = np.zeros((s.shape[0], 12), np.float32)
        out[:, :3] = s[:, :3]
        out[:, 3] = 1.0
        out[:, 4:7] = s[:, 4:7]
        out[:, 9] = s[:, 3]
        del clusters[:]
        order = np.argsort(lab, kind="stable")
        bounds = np.searchsorted(lab[order], np.arange(r["n_clusters"] + 1))
        for k in range(r["n_clusters"]):
            idx = order[bounds[k]:bounds[k + 1]]
            clusters.append(idx.astype(np.int32))
            out[idx, 8] = _cluster_rgb(k)
        return out
    kept = c.prefilter(cloud_in, params)
    if args and args[0] is not None:
        prev = np.asarray(args[0], np.float32).reshape(-1, 3)
        return np.concatenate([prev, kept], 0)
    return kept
