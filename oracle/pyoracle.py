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


# ---------------------------------------------------------------- App's stream ----------------
def transform_cloud(T, pts):
    """pcl::transformPointCloud (pcl 1.8 common/impl/transforms.hpp) in float: x' = ((r00 x +
    r01 y) + r02 z) + t0 per row, each operation rounded to float. T: 4x4 row-major."""
    T = np.asarray(T, np.float32)
    P = np.ascontiguousarray(pts, np.float32)[:, :3]
    out = np.empty_like(P)
    for r in range(3):
        s = T[r, 0] * P[:, 0]
        s = (s + T[r, 1] * P[:, 1]).astype(np.float32)
        s = (s + T[r, 2] * P[:, 2]).astype(np.float32)
        out[:, r] = (s + T[r, 3]).astype(np.float32)
    return out


def corrected_origin(T, prior_origin):
    """Translation of correction_iso * prior_pose (aligned_cloud.cpp:61-70) with
    correction_iso = fromMatrix4fToIsometry3d(T) (common.cpp:4-23): Eigen's Quaternionf of the
    float rotation block (trace branch / largest-diagonal branch), cast to double,
    toRotationMatrix in double, R * o + t with left-to-right row sums."""
    f = np.float32
    m = np.asarray(T, np.float32)[:3, :3]
    q = [f(0)] * 4  # x, y, z, w
    t = f(f(m[0, 0] + m[1, 1]) + m[2, 2])
    if t > f(0):
        t = f(np.sqrt(f(t + f(1))))
        q[3] = f(f(0.5) * t)
        t = f(f(0.5) / t)
        q[0] = f(f(m[2, 1] - m[1, 2]) * t)
        q[1] = f(f(m[0, 2] - m[2, 0]) * t)
        q[2] = f(f(m[1, 0] - m[0, 1]) * t)
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = f(np.sqrt(f(f(f(m[i, i] - m[j, j]) - m[k, k]) + f(1))))
        q[i] = f(f(0.5) * t)
        t = f(f(0.5) / t)
        q[3] = f(f(m[k, j] - m[j, k]) * t)
        q[j] = f(f(m[j, i] + m[i, j]) * t)
        q[k] = f(f(m[k, i] + m[i, k]) * t)
    x, y, z, w = (float(v) for v in q)
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    R = [[1.0 - (tyy + tzz), txy - twz, txz + twy],
         [txy + twz, 1.0 - (txx + tzz), tyz - twx],
         [txz - twy, tyz + twx, 1.0 - (txx + tyy)]]
    o = [float(v) for v in prior_origin]
    Tt = np.asarray(T, np.float32)
    return np.array([((R[r][0] * o[0] + R[r][1] * o[1]) + R[r][2] * o[2]) + float(Tt[r, 3]) for r in range(3)])


def mul4(A, B):
    """Eigen Matrix4f product A * B in float: each coefficient summed over k = 0..3 in order."""
    A = np.asarray(A, np.float32)
    B = np.asarray(B, np.float32)
    C = np.zeros((4, 4), np.float32)
    for r in range(4):
        for c in range(4):
            s = np.float32(A[r, 0] * B[0, c])
            for k in range(1, 4):
                s = np.float32(s + np.float32(A[r, k] * B[k, c]))
            C[r, c] = s
    return C


def sequence(first, first_origin, readings, origins, cfg=None, reference_update_frequency=5,
             max_correction_magnitude=1.0, resolution=0.2, overlap=True, stop=None, working_mode="robot",
             prefilter_with=None):
    """App::processCloud over a stream (app.cpp:282-414, robot mode): the first cloud is the
    reference; each reading: overlap -> ratio -> ICP against the current reference; dropped when
    some |T(i,3)| > max_correction_magnitude (float compare, app.cpp:366-373); an accepted reading
    is transformed by T and, as the reference_update_frequency-th accepted reading since the last
    update, becomes the reference with origin corrected_origin(T, its origin); a registration
    error ends the stream (app.cpp:210). stop: process only readings [0, stop).
    working_mode "debug" (app.cpp:87-96, 414): each reading is first transformed by initialT_
    (float, transform_cloud) and its prior pose becomes initialT_ * prior pose; after an accepted
    reading initialT_ = correction * initialT_ (a dropped reading returns before that line).
    prefilter_with (PrefilterParams, or True for the defaults): the clouds are RAW, in App's order:
    the first cloud is pre-filtered as given (app.cpp:293-297); a reading is moved by initialT_
    (debug mode) and then pre-filtered (setAndFilterReading, app.cpp:77-100). Each record then also
    holds n_kept, the reading's point count after the pre-filter.
    Returns a list of dicts (status, T, stats, accepted, reference, is_reference,
    corrected_origin, overlap, counts, ratio, prior_origin)."""
    cfg = cfg or default_config()
    pfp = None
    if prefilter_with is not None:
        pfp = prefilter_params() if prefilter_with is True else prefilter_with
        first = prefilter(first, pfp)["out"]
    ref, ref_origin, ref_id = _pts(first), np.asarray(first_origin, np.float64), -1
    acc = 0
    out = []
    mc = np.float32(max_correction_magnitude)
    initT = np.eye(4, dtype=np.float32)
    for i, (r, o) in enumerate(zip(readings, origins)):
        if stop is not None and i >= stop:
            break
        if working_mode == "debug":
            r = transform_cloud(initT, r)
            o = corrected_origin(initT, o)
        if pfp is not None:
            r = prefilter(r, pfp)["out"]
        rec = dict(reference=ref_id, is_reference=0, accepted=0, corrected_origin=None,
                   prior_origin=np.asarray(o, np.float64))
        if pfp is not None:
            rec["n_kept"] = len(r)
        if overlap:
            ov, cnt = globals()["overlap"](ref, ref_origin, r, o, resolution)
            ratio = autotune_ratio(ov)
            rec.update(overlap=ov, counts=cnt)
        else:
            ratio = cfg.trimmed_ratio
        c = IcpConfig.from_buffer_copy(cfg)
        c.trimmed_ratio = ratio
        rc, T, st = icp(ref, r, c)
        rec.update(status=rc, T=T, stats=st, ratio=ratio)
        out.append(rec)
        if rc:
            break
        Tf = np.asarray(T, np.float32)
        if any(abs(Tf[k, 3]) > mc for k in range(3)):
            continue
        rec["accepted"] = 1
        rec["corrected_origin"] = corrected_origin(Tf, o)
        acc += 1
        if acc == reference_update_frequency:
            ref, ref_origin, ref_id = transform_cloud(Tf, r), rec["corrected_origin"], i
            rec["is_reference"] = 1
            acc = 0
        initT = mul4(Tf, initT)
    return out
