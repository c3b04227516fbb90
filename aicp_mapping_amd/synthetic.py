"""Seeded synthetic lidar scenes for the benchmark configs of SURVEY.md §8(d).

The reference ships no clouds for its headline configs (the test data is external,
aicp_core/test/aicp_test.cpp:50-57), so inputs are synthetic with the §8(d) recipe:

* scene: ground z = 0 over 80 x 80 m, two walls y = +-6 m (4 m high), 40 random
  axis-aligned boxes with 0.5-3 m edges (seed);
* surfaces sampled on a jittered 0.08 m grid (the VoxelGrid leaf of
  aicp_core/src/utils/filteringUtils.cpp:12), Gaussian noise sigma = 0.01 m per axis;
* points kept within a 30 m box of the sensor origin (velodyne_accumulator.cpp:60) and
  subsampled to the nominal count, then ordered like a voxel-grid output (raster order);
* reading: same scene, independent sample (seed + 1), sensor origin moved 1.5 m,
  expressed through T_gt^-1 with T_gt = (yaw 2 deg, roll 0.5 deg, pitch -0.5 deg,
  t = (0.15, -0.10, 0.05) m).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np


def rot_zyx(yaw, pitch, roll):
    cy, sy = math.cos(yaw), math.sin(yaw)
    cp, sp = math.cos(pitch), math.sin(pitch)
    cr, sr = math.cos(roll), math.sin(roll)
    Rz = np.array([[cy, -sy, 0], [sy, cy, 0], [0, 0, 1]])
    Ry = np.array([[cp, 0, sp], [0, 1, 0], [-sp, 0, cp]])
    Rx = np.array([[1, 0, 0], [0, cr, -sr], [0, sr, cr]])
    return Rz @ Ry @ Rx


def make_T(yaw_deg=2.0, pitch_deg=-0.5, roll_deg=0.5, t=(0.15, -0.10, 0.05)):
    T = np.eye(4)
    T[:3, :3] = rot_zyx(math.radians(yaw_deg), math.radians(pitch_deg), math.radians(roll_deg))
    T[:3, 3] = t
    return T


T_GT = make_T()


@dataclass
class Scene:
    boxes: np.ndarray  # (B, 6): xmin, ymin, zmin, xmax, ymax, zmax


def make_scene(seed: int = 1, n_boxes: int = 40, extent: float = 40.0) -> Scene:
    rng = np.random.default_rng(seed)
    boxes = []
    while len(boxes) < n_boxes:
        e = rng.uniform(0.5, 3.0, size=3)
        c = rng.uniform(-extent + 2, extent - 2, size=2)
        if abs(c[1]) < 6.0 + e[1] / 2 and abs(c[1]) > 6.0 - e[1] / 2 - 0.5:
            continue  # keep boxes off the walls
        boxes.append([c[0] - e[0] / 2, c[1] - e[1] / 2, 0.0, c[0] + e[0] / 2, c[1] + e[1] / 2, e[2]])
    return Scene(np.asarray(boxes, np.float64))


def _grid(rng, u0, u1, v0, v1, spacing):
    us = np.arange(u0, u1, spacing)
    vs = np.arange(v0, v1, spacing)
    if us.size == 0 or vs.size == 0:
        return np.zeros((0, 2))
    U, V = np.meshgrid(us, vs, indexing="ij")
    P = np.stack([U.ravel(), V.ravel()], 1)
    P += rng.uniform(0, spacing, size=P.shape)
    keep = (P[:, 0] < u1) & (P[:, 1] < v1)
    return P[keep]


def sample_scene(scene: Scene, rng, origin, half=30.0, spacing=0.08, noise=0.01, extent=40.0):
    ox, oy = origin[0], origin[1]
    x0, x1 = max(-extent, ox - half), min(extent, ox + half)
    y0, y1 = max(-extent, oy - half), min(extent, oy + half)
    parts = []
    g = _grid(rng, x0, x1, y0, y1, spacing)  # ground
    parts.append(np.c_[g, np.zeros(len(g))])
    for wy in (-6.0, 6.0):  # walls
        if y0 <= wy <= y1:
            w = _grid(rng, x0, x1, 0.0, 4.0, spacing)
            parts.append(np.c_[w[:, 0], np.full(len(w), wy), w[:, 1]])
    for b in scene.boxes:
        bx0, by0, bz0, bx1, by1, bz1 = b
        if bx1 < x0 or bx0 > x1 or by1 < y0 or by0 > y1:
            continue
        t = _grid(rng, bx0, bx1, by0, by1, spacing)
        parts.append(np.c_[t, np.full(len(t), bz1)])
        for xx in (bx0, bx1):
            s = _grid(rng, by0, by1, bz0, bz1, spacing)
            parts.append(np.c_[np.full(len(s), xx), s])
        for yy in (by0, by1):
            s = _grid(rng, bx0, bx1, bz0, bz1, spacing)
            parts.append(np.c_[s[:, 0], np.full(len(s), yy), s[:, 1]])
    P = np.concatenate(parts, 0)
    P += rng.normal(0, noise, size=P.shape)
    m = (np.abs(P[:, 0] - ox) <= half) & (np.abs(P[:, 1] - oy) <= half)
    return P[m]


def _subsample_raster(P, n, rng, leaf=0.08):
    if n < len(P):
        P = P[rng.choice(len(P), size=n, replace=False)]
    k = np.floor(P / leaf).astype(np.int64)
    k -= k.min(0)
    order = np.lexsort((k[:, 2], k[:, 1], k[:, 0]))
    return P[order]


@dataclass
class Pair:
    ref: np.ndarray  # (M, 3) float32
    read: np.ndarray  # (N, 3) float32
    ref_origin: np.ndarray  # (3,) float64
    read_origin: np.ndarray  # (3,) float64, in the reading's frame
    T_gt: np.ndarray  # 4x4, ref ~ T_gt * read


def make_pair(n_ref: int, n_read: int, seed: int = 1, T_gt=None, move=1.5, sensor_z=0.7,
              half=30.0) -> Pair:
    T_gt = T_GT if T_gt is None else np.asarray(T_gt, np.float64)
    scene = make_scene(seed)
    o_ref = np.array([0.0, 0.0, sensor_z])
    o_read_w = np.array([move, 0.0, sensor_z])
    rng_r = np.random.default_rng(seed * 7919 + 1)
    rng_d = np.random.default_rng(seed * 7919 + 2)
    ref = _subsample_raster(sample_scene(scene, rng_r, o_ref, half=half), n_ref, rng_r)
    read_w = _subsample_raster(sample_scene(scene, rng_d, o_read_w, half=half), n_read, rng_d)
    Ti = np.linalg.inv(T_gt)
    read = read_w @ Ti[:3, :3].T + Ti[:3, 3]
    o_read = Ti[:3, :3] @ o_read_w + Ti[:3, 3]
    return Pair(ref.astype(np.float32), read.astype(np.float32), o_ref, o_read, T_gt)


def make_sequence(n_readings: int = 64, ref_every: int = 5, n_points: int = 120000, seed: int = 1,
                  step: float = 0.3, sensor_z: float = 0.7, half: float = 30.0, T_gt=None) -> list:
    """C2 of SURVEY.md §8(d): a streamed sequence of readings registered frame-to-reference,
    the reference replaced every `ref_every` readings (aicp.launch reference_update_frequency
    5). Reading i is taken `step` m further along x than reading i-1 and is perturbed by T_gt;
    reading i is paired with reference i // ref_every, and pairs of one window share the SAME
    reference array (the C-ABI then builds its kd-tree and normals once)."""
    T_gt = T_GT if T_gt is None else np.asarray(T_gt, np.float64)
    scene = make_scene(seed)
    Ti = np.linalg.inv(T_gt)
    refs, pairs = [], []
    for i in range(n_readings):
        j = i // ref_every
        if j == len(refs):
            o_ref = np.array([j * ref_every * step, 0.0, sensor_z])
            rng_r = np.random.default_rng(seed * 7919 + 1000 + j)
            ref = _subsample_raster(sample_scene(scene, rng_r, o_ref, half=half), n_points, rng_r)
            refs.append((ref.astype(np.float32), o_ref))
        ref, o_ref = refs[j]
        o_read_w = np.array([(i + 1) * step, 0.0, sensor_z])
        rng_d = np.random.default_rng(seed * 7919 + 5000 + i)
        read_w = _subsample_raster(sample_scene(scene, rng_d, o_read_w, half=half), n_points, rng_d)
        read = (read_w @ Ti[:3, :3].T + Ti[:3, 3]).astype(np.float32)
        o_read = Ti[:3, :3] @ o_read_w + Ti[:3, 3]
        pairs.append(Pair(ref, read, o_ref, o_read, T_gt))
    return pairs


@dataclass
class Stream:
    first: np.ndarray          # the first cloud (App's first reference), world frame
    first_origin: np.ndarray   # its sensor origin
    readings: list             # reading clouds in their drifted (odometry) frame
    origins: list              # prior-pose translations (sensor origins) in that frame
    T_gt: list                 # correction that re-aligns each reading (drift^-1)


def make_stream(n_readings: int = 64, n_points: int = 120000, seed: int = 1, step: float = 0.3,
                sensor_z: float = 0.7, half: float = 30.0, T_gt=None, jumps=None) -> Stream:
    """The input of App's frame-to-reference stream (app.cpp:282-414) for the C2/C3 configs of
    SURVEY.md §8(d): a first cloud at the start of the path, then readings taken `step` m apart
    along x, each perturbed by the odometry drift T_gt^-1. Unlike make_sequence, references are
    not sampled here: App builds them from the corrected readings. jumps: {reading index: extra
    translation (3,)} of that reading's drift, to make App drop it (max_correction_magnitude)."""
    first, o0 = stream_first(seed, n_points, sensor_z, half)
    out = [stream_reading(seed, i, n_points, step, sensor_z, half, T_gt, (jumps or {}).get(i))
           for i in range(n_readings)]
    return Stream(first, o0, [r[0] for r in out], [r[1] for r in out], [r[2] for r in out])


def stream_first(seed: int, n_points: int, sensor_z: float = 0.7, half: float = 30.0):
    """make_stream's first cloud and its origin."""
    o0 = np.array([0.0, 0.0, sensor_z])
    rng0 = np.random.default_rng(seed * 7919 + 1000)
    first = _subsample_raster(sample_scene(make_scene(seed), rng0, o0, half=half), n_points, rng0)
    return first.astype(np.float32), o0


def stream_reading(seed: int, i: int, n_points: int, step: float = 0.3, sensor_z: float = 0.7, half: float = 30.0,
                   T_gt=None, jump=None):
    """make_stream's reading i: (points, origin, T_gt) (independent of the others, so a process
    pool can build a stream)."""
    Tg = (T_GT if T_gt is None else np.asarray(T_gt, np.float64)).copy()
    if jump is not None:
        Tg[:3, 3] += np.asarray(jump, np.float64)
    Ti = np.linalg.inv(Tg)
    o_w = np.array([(i + 1) * step, 0.0, sensor_z])
    rng = np.random.default_rng(seed * 7919 + 5000 + i)
    w = _subsample_raster(sample_scene(make_scene(seed), rng, o_w, half=half), n_points, rng)
    return (w @ Ti[:3, :3].T + Ti[:3, 3]).astype(np.float32), Ti[:3, :3] @ o_w + Ti[:3, 3], Tg


def make_cube(min_corner=-2.0, max_corner=2.0, step=0.05):
    """The cube of aicp_core/src/tools/create_cube_cloud.cpp:13-90 (float loop counters)."""
    vals = []
    i = np.float32(min_corner)
    while i < np.float32(max_corner):
        vals.append(i)
        i = np.float32(i + np.float32(step))
    v = np.asarray(vals, np.float32)
    I, J = np.meshgrid(v, v, indexing="ij")
    I, J = I.ravel(), J.ravel()
    lo = np.full_like(I, np.float32(min_corner))
    hi = np.full_like(I, np.float32(max_corner))
    faces = [
        np.c_[I, J, lo], np.c_[I, J, hi],  # bottom, top
        np.c_[lo, I, J], np.c_[hi, I, J],  # side A, B
        np.c_[I, lo, J], np.c_[I, hi, J],  # side C, D
    ]
    return np.concatenate(faces, 0).astype(np.float32)


def transform(T, P):
    T = np.asarray(T, np.float64)
    return (np.asarray(P, np.float64) @ T[:3, :3].T + T[:3, 3]).astype(np.float32)


def rot_err(Ta, Tb):
    """compute_transl_rot_errors_from_transform.py:36-43: acos((tr dR - 1)/2) of Ta^-1 Tb."""
    D = np.linalg.inv(np.asarray(Ta, np.float64)) @ np.asarray(Tb, np.float64)
    c = np.clip((np.trace(D[:3, :3]) - 1) / 2, -1.0, 1.0)
    return float(math.acos(c)), float(np.linalg.norm(D[:3, 3]))
