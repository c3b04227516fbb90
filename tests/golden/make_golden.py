#!/usr/bin/env python3
"""Generate tests/golden/*.npz: small input/expected-output vectors for every hot-path row.

The expected outputs come from the CPU oracle (oracle/, the restatement of the
libpointmatcher / libnabo / octomap chain; parity unpinned). They pin the
oracle itself against drift (tests/test_golden.py, CPU) and the device against them
(tests/test_golden.py, -m gpu). Inputs are the SURVEY §8(c) cases at fixture size:
  (1) a planar 2-D scan lifted to 3-D (z = 0: rank-deficient point-to-plane) and its extruded
      variant (21 z layers), synthesised here since the reference's scan CSVs are not copied;
  (2) the cube of create_cube_cloud.cpp with the registration_main.cpp perturbation recipe;
  (3) seeded synthetic planar scenes (§8(d)) at <= 5k points.
Regenerate: python tests/golden/make_golden.py   (deterministic; numpy only plus the oracle)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import pyoracle as po  # noqa: E402
from aicp_mapping_amd import synthetic as sy  # noqa: E402

RES = float(np.float32(0.2))


def scan2d(seed, n=2162):
    """A room-like 2-D laser scan (walls + a few pillars), z = 0."""
    rng = np.random.default_rng(seed)
    ang = np.sort(rng.uniform(-np.pi, np.pi, n))
    r = np.full(n, 6.0)
    r = np.minimum(r, np.abs(4.0 / np.cos(ang)))  # walls x = +-4
    r = np.minimum(r, np.abs(3.0 / np.sin(ang)))  # walls y = +-3
    for cx, cy in [(1.5, 1.0), (-2.0, -1.2)]:
        d = cx * np.cos(ang) + cy * np.sin(ang)
        disc = d * d - (cx * cx + cy * cy - 0.09)
        hit = (disc > 0) & (d > 0)
        r = np.where(hit, np.minimum(r, d - np.sqrt(np.maximum(disc, 0))), r)
    r = r + rng.normal(0, 0.01, n)
    return np.c_[r * np.cos(ang), r * np.sin(ang), np.zeros(n)].astype(np.float32)


def extrude(p, layers=21, height=2.0):
    """21 z-layers over 0-2 m plus a floor (here over a 600-point scan)."""
    zs = np.linspace(0.0, height, layers, dtype=np.float32)
    out = np.concatenate([np.c_[p[:, :2], np.full(len(p), z, np.float32)] for z in zs])
    xs = np.linspace(-4, 4, 41, dtype=np.float32)
    ys = np.linspace(-3, 3, 31, dtype=np.float32)
    fx, fy = np.meshgrid(xs, ys)
    floor = np.c_[fx.ravel(), fy.ravel(), np.zeros(fx.size, np.float32)]
    return np.concatenate([out, floor]).astype(np.float32)


def icp_case(ref, read, ratio, T0=None):
    cfg = po.default_config(trimmed_ratio=ratio)
    rc, T, st = po.icp(ref, read, cfg, T0=T0)
    return dict(rc=np.int32(rc), T=T.astype(np.float32), iterations=np.int32(st.iterations),
                inlier_ratio=np.float32(st.inlier_ratio))


def main():
    po.lib()
    # --- kd-tree NN (libnabo order): synthetic scene + duplicates
    pr = sy.make_pair(4000, 1000, seed=21, half=15.0)
    ref = pr.ref.copy()
    ref[100:140] = ref[100]
    tree = po.Tree(ref)
    ids1, d21, tp1, tn1 = tree.knn(pr.read, k=1, eps=3.16)
    ids20, d220, tp20, tn20 = tree.knn(ref[:500], k=20, eps=0.0)
    np.savez_compressed(os.path.join(HERE, "knn.npz"), ref=ref, queries=pr.read, ids_k1_eps316=ids1,
                        d2_k1_eps316=d21, touched_k1=np.array([tp1, tn1], np.uint64), ids_k20=ids20,
                        d2_k20=d220, touched_k20=np.array([tp20, tn20], np.uint64))
    # --- SurfaceNormal (knn 20) incl. a degenerate line
    pts = np.concatenate([ref[:3000], np.c_[np.linspace(0, 1, 40), np.zeros(40), np.zeros(40)].astype(np.float32)])
    nrm, dens, deg = po.surface_normals(pts, 20)
    np.savez_compressed(os.path.join(HERE, "normals.npz"), pts=pts, normals=nrm, degenerate=np.int32(deg))
    # --- trimmed quantile
    rng = np.random.default_rng(5)
    d2 = (rng.random(7777) ** 3).astype(np.float32)
    d2[::97] = np.inf
    qs = np.array([0.25, 0.358818, 0.5, 0.7, 1.0], np.float32)
    lim = np.array([po.dists_quantile(d2, float(q))[0] for q in qs], np.float32)
    np.savez_compressed(os.path.join(HERE, "quantile.npz"), d2=d2, ratios=qs, limits=lim)
    # --- 6x6 solves: full rank, rank 3 (planar), rank 5
    As, bs, xs, paths = [], [], [], []
    for r in (6, 5, 3):
        M = rng.normal(size=(6, r))
        A = M @ M.T
        b = A @ rng.normal(size=6)
        x, path = po.solve6(A, b)
        As.append(A), bs.append(b), xs.append(x), paths.append(path)
    np.savez_compressed(os.path.join(HERE, "solve6.npz"), A=np.array(As), b=np.array(bs), x=np.array(xs),
                        path=np.array(paths, np.int32))
    # --- overlap (octree-equivalent key sets) and the ratio rule
    pr = sy.make_pair(3000, 3000, seed=22, half=12.0)
    ov, cnt = po.overlap(pr.ref, pr.ref_origin, pr.read, pr.read_origin, RES)
    np.savez_compressed(os.path.join(HERE, "overlap.npz"), ref=pr.ref, read=pr.read, ref_origin=pr.ref_origin,
                        read_origin=pr.read_origin, resolution=np.float64(RES), counts=cnt,
                        overlap=np.float32(ov), ratio=np.float32(po.autotune_ratio(ov)))
    # --- whole ICP: lifted 2-D scans (rank-deficient), extruded scans, cube recipe, scene
    cases = {}
    s0 = scan2d(0)
    Tg = sy.make_T(yaw_deg=3.0, pitch_deg=0.0, roll_deg=0.0, t=(0.1, -0.05, 0.0))
    cases["scan_lifted"] = (s0, sy.transform(np.linalg.inv(Tg), s0).astype(np.float32), 0.7, None)
    e0 = extrude(s0[::4])
    cases["scan_extruded"] = (e0, sy.transform(np.linalg.inv(Tg), e0).astype(np.float32), 0.6, None)
    cube = sy.make_cube()
    rng = np.random.default_rng(3)
    Tc = sy.make_T(yaw_deg=rng.normal(0, 1.0), pitch_deg=0, roll_deg=0,
                   t=(rng.normal(0, 0.1), rng.normal(0, 0.1), 0.0))
    cases["cube"] = (cube, sy.transform(np.linalg.inv(Tc), cube).astype(np.float32), 0.7, None)
    cube_T = Tc.astype(np.float64)
    pr = sy.make_pair(5000, 5000, seed=23, half=15.0)
    cases["scene"] = (pr.ref, pr.read, 0.5, None)
    T0 = sy.make_T(yaw_deg=1.0, pitch_deg=0.0, roll_deg=0.0, t=(0.05, 0.0, 0.0)).astype(np.float32)
    cases["scene_T0"] = (pr.ref, pr.read, 0.5, T0)
    arrays = {"cube__perturbation": cube_T}
    for name, (r, d, ratio, t0) in cases.items():
        res = icp_case(r, d, ratio, t0)
        if name != "cube":  # the cube and its reading are regenerated (synthetic.make_cube)
            arrays[f"{name}__ref"] = r
            arrays[f"{name}__read"] = d
        arrays[f"{name}__ratio"] = np.float32(ratio)
        arrays[f"{name}__T0"] = np.eye(4, dtype=np.float32) if t0 is None else t0
        for k, v in res.items():
            arrays[f"{name}__{k}"] = v
    np.savez_compressed(os.path.join(HERE, "icp.npz"), names=np.array(list(cases)), **arrays)
    for f in sorted(os.listdir(HERE)):
        if f.endswith(".npz"):
            print(f, os.path.getsize(os.path.join(HERE, f)))


if __name__ == "__main__":
    main()
