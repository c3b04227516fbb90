"""Localization-only map crop: getPointsInOrientedBox,
aicp_core/src/utils/filteringUtils.cpp:619-637, pcl::CropBox around the prior pose.

CPU: the oracle's Eigen eulerAngles(0,1,2) restatement reproduces the rotation, and the crop
matches an independent float64 numpy restatement away from the box faces. GPU: the device crop
is bit-exact (same points, same order) with the oracle, including NaNs, empty and ragged tile
sizes, and at C4 map size (~690k points). Parity against PCL itself is unpinned (PCL and
Eigen are not in the image; no reference fixture covers the crop).
"""
import math

import numpy as np
import pytest

from aicp_mapping_amd import synthetic as sy


def Rx(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[1, 0, 0], [0, c, -s], [0, s, c]])


def Ry(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, 0, s], [0, 1, 0], [-s, 0, c]])


def Rz(a):
    c, s = math.cos(a), math.sin(a)
    return np.array([[c, -s, 0], [s, c, 0], [0, 0, 1]])


def pose(yaw, pitch, roll, t):
    T = np.eye(4)
    T[:3, :3] = Rz(yaw) @ Ry(pitch) @ Rx(roll)
    T[:3, 3] = t
    return T


POSES = [np.eye(4), pose(0.0, 0.0, 0.0, (3.0, -2.0, 0.5)), pose(0.7, 0.0, 0.0, (1.0, 2.0, 0.0)),
         pose(-2.5, 0.1, -0.05, (-4.0, 0.3, 1.0)), pose(1.2, -0.4, 0.9, (0.0, 0.0, 0.0))]


def numpy_crop(P, mn, mx, T, rpy):
    """Float64 restatement: local = (Rz Ry Rx)(rpy)^T (p - t), inclusive cube test."""
    R = Rz(rpy[2]) @ Ry(rpy[1]) @ Rx(rpy[0])
    L = (P.astype(np.float64) - T[:3, 3]) @ R
    keep = np.all((L >= mn) & (L <= mx), axis=1) & np.all(np.isfinite(P), axis=1)
    return keep, L


@pytest.mark.parametrize("T", POSES)
def test_oracle_euler_angles_reproduce_rotation(oracle, T):
    _, rpy = oracle.crop_box(np.zeros((1, 3), np.float32), -1, 1, T)
    R = Rx(rpy[0]) @ Ry(rpy[1]) @ Rz(rpy[2])  # eulerAngles(0,1,2): R = Rx Ry Rz
    assert np.allclose(R, T[:3, :3], atol=1e-5)
    assert 0.0 <= -rpy[0] + math.pi + 1e-6 and rpy[0] <= math.pi + 1e-6


@pytest.mark.parametrize("T", POSES)
def test_oracle_crop_matches_numpy_away_from_faces(oracle, T):
    P = np.random.default_rng(4).uniform(-25, 25, size=(20000, 3)).astype(np.float32)
    kept, rpy = oracle.crop_box(P, -15.0, 15.0, T)
    keep, L = numpy_crop(P, -15.0, 15.0, T, rpy.astype(np.float64))
    margin = np.min(np.abs(np.concatenate([L + 15.0, L - 15.0], axis=1)), axis=1)
    clear = margin > 1e-4
    kept_set = {tuple(p) for p in kept.tolist()}
    got = np.array([tuple(p) in kept_set for p in P.tolist()])
    assert np.array_equal(got[clear], keep[clear])
    # input order preserved
    idx = np.flatnonzero(got)
    assert np.array_equal(kept, P[idx])


def test_oracle_crop_drops_nonfinite(oracle):
    P = np.array([[0, 0, 0], [np.nan, 0, 0], [1, np.inf, 0], [2, 2, 2], [20, 0, 0]], np.float32)
    kept, _ = oracle.crop_box(P, -15, 15, np.eye(4))
    assert np.array_equal(kept, P[[0, 3]])


@pytest.mark.gpu
@pytest.mark.parametrize("n", [0, 1, 1023, 1024, 1025, 70001])
@pytest.mark.parametrize("k", range(len(POSES)))
def test_crop_box_bit_exact(oracle, n, k):
    import aicp_mapping_amd._lib as L

    rng = np.random.default_rng(n + 17 * k)
    P = rng.uniform(-25, 25, size=(n, 3)).astype(np.float32)
    if n > 10:
        P[rng.integers(0, n, 5)] = np.nan
    ctx = L.Context(0)
    try:
        got, rpy = ctx.crop_box(P, -15.0, 15.0, POSES[k])
    finally:
        ctx.close()
    exp, rpy1 = oracle.crop_box(P, -15.0, 15.0, POSES[k])
    assert np.array_equal(rpy, rpy1)
    assert got.shape == exp.shape and np.array_equal(got, exp)


@pytest.mark.gpu
def test_crop_box_c4_map_size(oracle):
    """C4-size map (make_pair asks for 1M points; 688 682 remain inside its 30 m sampling box)
    cropped to +-15 m around a prior pose (app.cpp:41-51)."""
    import aicp_mapping_amd._lib as L

    pr = sy.make_pair(1_000_000, 10, seed=8)
    T = pose(0.3, 0.0, 0.0, pr.ref_origin)
    ctx = L.Context(0)
    try:
        got, _ = ctx.crop_box(pr.ref, -15.0, 15.0, T)
    finally:
        ctx.close()
    exp, _ = oracle.crop_box(pr.ref, -15.0, 15.0, T)
    assert 0 < len(exp) < len(pr.ref) and np.array_equal(got, exp)


def test_bench_c4_crop_is_reference_crop(oracle):
    """bench.py's C4 input preparation (axis-aligned +-15 m box around the prior position)
    equals getPointsInOrientedBox with an identity-rotation pose, point for point."""
    P = np.random.default_rng(12).uniform(-40, 40, size=(50000, 3)).astype(np.float32)
    o = np.array([0.9, 0.0, 0.7])
    m = np.all(np.abs(P - o.astype(np.float32)) <= 15.0, axis=1)
    T = np.eye(4)
    T[:3, 3] = o
    kept, rpy = oracle.crop_box(P, -15.0, 15.0, T)
    assert not np.any(rpy) and np.array_equal(kept, P[m])
