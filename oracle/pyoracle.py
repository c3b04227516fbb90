"""ctypes wrapper of the CPU oracle (oracle/libaicp_oracle.so) — TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module, and
only as the checker / the CPU baseline. Parity at the libpointmatcher boundary is UNPINNED
(see aicp_oracle.h and DESIGN.md).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libaicp_oracle.so")


def build(force: bool = False) -> str:
    srcs = [os.path.join(HERE, f) for f in ("aicp_oracle.cpp", "prefilter_oracle.cpp", "aicp_oracle.h")]
    if force or not os.path.exists(LIB_PATH) or any(os.path.getmtime(LIB_PATH) < os.path.getmtime(f) for f in srcs):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


class IcpConfig(C.Structure):
    _fields_ = [
        ("knn_normals", C.c_int32),
        ("nn_epsilon", C.c_float),
        ("nn_max_dist", C.c_float),
        ("trimmed_ratio", C.c_float),
        ("max_iter", C.c_int32),
        ("min_diff_rot", C.c_float),
        ("min_diff_trans", C.c_float),
        ("smooth_length", C.c_int32),
        ("bucket_size", C.c_int32),
        ("normals_on_centered", C.c_int32),
    ]


TRACE = 64


class IcpStats(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("iterations", C.c_int32),
        ("converged", C.c_int32),
        ("degenerate_normals", C.c_int32),
        ("inlier_ratio", C.c_float),
        ("mean", C.c_float * 3),
        ("tree_depth", C.c_int32),
        ("tree_nodes", C.c_int32),
        ("nn_points_touched", C.c_uint64),
        ("nn_nodes_touched", C.c_uint64),
        ("limit", C.c_float * TRACE),
        ("kept", C.c_int32 * TRACE),
        ("solve_path", C.c_int32 * TRACE),
        ("T_iter", (C.c_float * 16) * TRACE),
        ("A0", C.c_double * 36),
        ("b0", C.c_double * 6),
    ]


def default_config(**kw) -> IcpConfig:
    """icp_autotuned_default.yaml:9-51 (ratio 0.70 before auto-tune)."""
    c = IcpConfig(20, 3.16, float("inf"), 0.70, 20, 0.001, 0.01, 4, 8, 0)
    for k, v in kw.items():
        setattr(c, k, v)
    return c


class PrefilterParams(C.Structure):
    _fields_ = [
        ("leaf", C.c_float),
        ("normal_k", C.c_int32),
        ("neighbours", C.c_int32),
        ("min_cluster", C.c_int32),
        ("max_cluster", C.c_int32),
        ("cos_smoothness", C.c_float),
        ("curvature", C.c_float),
        ("viewpoint", C.c_float * 3),
    ]


def prefilter_params(leaf=0.08, normal_k=30, neighbours=15, min_cluster=50, max_cluster=1000000,
                     smoothness_rad=3.0 / 180.0 * np.pi, curvature=1.0, viewpoint=(0.0, 0.0, 0.0)):
    """filteringUtils.cpp:12,22,27-34. validatePoint compares with cosf(theta) of the float theta."""
    cos_s = np.float32(np.cos(np.float64(np.float32(smoothness_rad))))
    return PrefilterParams(leaf, normal_k, neighbours, min_cluster, max_cluster, float(cos_s), curvature,
                           (C.c_float * 3)(*viewpoint))


_lib = None


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        fp = C.POINTER(C.c_float)
        dp = C.POINTER(C.c_double)
        ip = C.POINTER(C.c_int32)
        up = C.POINTER(C.c_uint64)
        vp = C.c_void_p
        L.ao_tree_build.argtypes = [fp, C.c_int64, C.c_int64, C.c_int, C.POINTER(vp)]
        L.ao_tree_free.argtypes = [vp]
        L.ao_tree_info.argtypes = [vp, ip, ip, ip]
        L.ao_tree_export.argtypes = [vp, ip, fp, ip, ip, ip]
        L.ao_tree_knn.argtypes = [vp, fp, C.c_int64, C.c_int64, C.c_int, C.c_float, C.c_int,
                                  C.c_float, ip, fp, up, up]
        L.ao_partition_sequential.argtypes = [fp, ip, C.c_int32, C.c_float, ip, ip]
        L.ao_partition_parallel.argtypes = [fp, ip, C.c_int32, C.c_float, ip, ip]
        L.ao_surface_normals.argtypes = [fp, C.c_int64, C.c_int64, C.c_int, fp, fp, ip]
        L.ao_dists_quantile.argtypes = [fp, C.c_int64, C.c_float, ip]
        L.ao_dists_quantile.restype = C.c_float
        L.ao_solve6.argtypes = [dp, dp, dp, ip]
        L.ao_icp.argtypes = [fp, C.c_int64, C.c_int64, fp, C.c_int64, C.c_int64, fp,
                             C.POINTER(IcpConfig), fp, C.POINTER(IcpStats)]
        L.ao_overlap.argtypes = [fp, C.c_int64, C.c_int64, dp, fp, C.c_int64, C.c_int64, dp,
                                 C.c_double, fp, up]
        L.ao_ray_keys.argtypes = [fp, fp, C.c_double, up, C.c_int64]
        L.ao_ray_keys.restype = C.c_int64
        L.ao_autotune_ratio.argtypes = [C.c_float]
        L.ao_autotune_ratio.restype = C.c_float
        L.ao_quantize_ratio.argtypes = [C.c_float]
        L.ao_quantize_ratio.restype = C.c_float
        L.ao_crop_box.argtypes = [fp, C.c_int64, C.c_int64, C.c_float, C.c_float, fp, fp,
                                  C.POINTER(C.c_int64), fp]
        L.ao_prefilter.argtypes = [fp, C.c_int64, C.c_int64, C.POINTER(PrefilterParams), fp, ip,
                                   C.POINTER(C.c_int64), C.POINTER(C.c_int64), fp, C.POINTER(C.c_int64)]
        _lib = L
    return _lib


def _f(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _pts(p):
    p = np.ascontiguousarray(p, dtype=np.float32)
    assert p.ndim == 2 and p.shape[1] >= 3
    return p


class Tree:
    def __init__(self, pts, bucket=8):
        self.pts = _pts(pts)
        h = C.c_void_p()
        rc = lib().ao_tree_build(_f(self.pts), self.pts.shape[0], self.pts.shape[1], bucket, C.byref(h))
        assert rc == 0
        self.h = h

    def __del__(self):
        if getattr(self, "h", None):
            lib().ao_tree_free(self.h)
            self.h = None

    def info(self):
        n, d, lv = C.c_int32(), C.c_int32(), C.c_int32()
        lib().ao_tree_info(self.h, C.byref(n), C.byref(d), C.byref(lv))
        return n.value, d.value, lv.value

    def export(self):
        n, _, _ = self.info()
        cd = np.zeros(n, np.int32)
        cut = np.zeros(n, np.float32)
        roc = np.zeros(n, np.int32)
        bs = np.zeros(n, np.int32)
        bid = np.zeros(self.pts.shape[0], np.int32)
        ip = lambda a: a.ctypes.data_as(C.POINTER(C.c_int32))
        lib().ao_tree_export(self.h, ip(cd), _f(cut), ip(roc), ip(bs), ip(bid))
        return dict(cd=cd, cut=cut, right_or_count=roc, bucket_start=bs, bucket_ids=bid)

    def knn(self, q, k=1, eps=0.0, allow_self=True, max_radius=float("inf")):
        q = _pts(q)
        nq = q.shape[0]
        ids = np.zeros((nq, k), np.int32)
        d2 = np.zeros((nq, k), np.float32)
        tp, tn = C.c_uint64(0), C.c_uint64(0)
        lib().ao_tree_knn(self.h, _f(q), nq, q.shape[1], k, eps, int(allow_self), max_radius,
                          ids.ctypes.data_as(C.POINTER(C.c_int32)), _f(d2), C.byref(tp), C.byref(tn))
        return ids, d2, tp.value, tn.value


def partition(v, cut, parallel=False):
    v = np.ascontiguousarray(v, np.float32).copy()
    idx = np.arange(len(v), dtype=np.int32)
    b1, b2 = C.c_int32(), C.c_int32()
    fn = lib().ao_partition_parallel if parallel else lib().ao_partition_sequential
    fn(_f(v), idx.ctypes.data_as(C.POINTER(C.c_int32)), len(v), cut, C.byref(b1), C.byref(b2))
    return v, idx, b1.value, b2.value


def surface_normals(pts, knn=20):
    p = _pts(pts)
    n = p.shape[0]
    nrm = np.zeros((n, 3), np.float32)
    dens = np.zeros(n, np.float32)
    deg = C.c_int32()
    rc = lib().ao_surface_normals(_f(p), n, p.shape[1], knn, _f(nrm), _f(dens), C.byref(deg))
    assert rc == 0
    return nrm, dens, deg.value


def dists_quantile(d2, q):
    d2 = np.ascontiguousarray(d2, np.float32)
    err = C.c_int32()
    v = lib().ao_dists_quantile(_f(d2), d2.size, q, C.byref(err))
    return v, err.value


def solve6(A, b):
    A = np.ascontiguousarray(A, np.float64).reshape(6, 6)
    b = np.ascontiguousarray(b, np.float64).reshape(6)
    x = np.zeros(6, np.float64)
    path = C.c_int32()
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    lib().ao_solve6(dp(A), dp(b), dp(x), C.byref(path))
    return x, path.value


def icp(ref, read, cfg=None, T0=None):
    ref = _pts(ref)
    read = _pts(read)
    cfg = cfg or default_config()
    T = np.zeros(16, np.float32)
    st = IcpStats()
    t0p = None
    if T0 is not None:
        T0 = np.ascontiguousarray(np.asarray(T0, np.float32).reshape(4, 4).T.reshape(16))
        t0p = _f(T0)
    rc = lib().ao_icp(_f(ref), ref.shape[0], ref.shape[1], _f(read), read.shape[0], read.shape[1],
                      t0p, C.byref(cfg), _f(T), C.byref(st))
    return rc, T.reshape(4, 4).T.copy(), st  # row-major 4x4 for numpy


def overlap(ref, ref_origin, read, read_origin, resolution):
    ref = _pts(ref)
    read = _pts(read)
    ro = np.ascontiguousarray(ref_origin, np.float64)
    do = np.ascontiguousarray(read_origin, np.float64)
    out = C.c_float()
    cnt = np.zeros(3, np.uint64)
    dp = lambda a: a.ctypes.data_as(C.POINTER(C.c_double))
    rc = lib().ao_overlap(_f(ref), ref.shape[0], ref.shape[1], dp(ro), _f(read), read.shape[0],
                          read.shape[1], dp(do), resolution, C.byref(out),
                          cnt.ctypes.data_as(C.POINTER(C.c_uint64)))
    assert rc == 0
    return out.value, cnt


def ray_keys(origin, end, resolution, cap=100000):
    o = np.ascontiguousarray(origin, np.float32)
    e = np.ascontiguousarray(end, np.float32)
    out = np.zeros(cap, np.uint64)
    n = lib().ao_ray_keys(_f(o), _f(e), resolution, out.ctypes.data_as(C.POINTER(C.c_uint64)), cap)
    return None if n < 0 else out[:n].copy()


def autotune_ratio(overlap_percent):
    return lib().ao_autotune_ratio(overlap_percent)


def quantize_ratio(r):
    return lib().ao_quantize_ratio(r)


def crop_box(pts, mn, mx, origin):
    """getPointsInOrientedBox restatement (filteringUtils.cpp:619-637): (kept xyz, rpy)."""
    p = _pts(pts)
    o = np.ascontiguousarray(np.asarray(origin, np.float32).reshape(4, 4).T.reshape(16))
    out = np.zeros((p.shape[0], 3), np.float32)
    m = C.c_int64(0)
    rpy = np.zeros(3, np.float32)
    rc = lib().ao_crop_box(_f(p), p.shape[0], p.shape[1], mn, mx, _f(o), _f(out), C.byref(m), _f(rpy))
    assert rc == 0
    return out[:m.value].copy(), rpy


def prefilter(pts, params=None):
    """regionGrowingUniformPlaneSegmentationFilter (filteringUtils.cpp:5-45, 51-103) on the CPU.
    Returns dict(out=(n_out, 3) kept points, clusters concatenated; sampled=(V, 8) {x, y, z,
    curvature, nx, ny, nz, cluster}; labels=(V,) cluster or -1; n_clusters)."""
    p = _pts(pts)
    n = p.shape[0]
    prm = params or prefilter_params()
    sampled = np.zeros((max(n, 1), 8), np.float32)
    labels = np.zeros(max(n, 1), np.int32)
    out = np.zeros((max(n, 1), 3), np.float32)
    ns, nc, no = C.c_int64(), C.c_int64(), C.c_int64()
    rc = lib().ao_prefilter(_f(p), n, p.shape[1], C.byref(prm), _f(sampled),
                            labels.ctypes.data_as(C.POINTER(C.c_int32)), C.byref(ns), C.byref(nc), _f(out),
                            C.byref(no))
    if rc:
        raise RuntimeError(f"ao_prefilter failed ({rc})")
    V = ns.value
    return dict(out=out[:no.value].copy(), sampled=sampled[:V].copy(), labels=labels[:V].copy(),
                n_clusters=nc.value)
