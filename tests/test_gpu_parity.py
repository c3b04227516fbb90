"""Device parity tests: every hot-path kernel through the C-ABI against the CPU oracle.

Bar: bit-exact for index/integer work (NN ids, d^2 of the same float queries,
trimmed limit, overlap key counts), tolerance for floating-point results: transforms within
1e-4 rad / 1e-3 m of the oracle (north star), tighter (1e-6 rad / 1e-5 m) against the oracle
run with the device's normal-estimation layout.
"""
import math

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from aicp_mapping_amd import synthetic as sy

RES = float(np.float32(0.2))
ROT_TOL, TRANS_TOL = 1e-4, 1e-3


@pytest.fixture(scope="module")
def L():
    import aicp_mapping_amd._lib as L

    return L


@pytest.fixture(scope="module")
def ctx(L):
    c = L.Context(0)
    yield c
    c.close()


def rand_cloud(n, seed, scale=10.0):
    return np.random.default_rng(seed).uniform(-scale, scale, size=(n, 3)).astype(np.float32)


# ---------------------------------------------------------------- NN kernel ---------------
@pytest.mark.parametrize("k,eps", [(1, 0.0), (1, 3.16), (4, 0.0), (20, 0.0), (1, 0.5)])
def test_knn_bit_exact(ctx, oracle, k, eps):
    pts = rand_cloud(20000, 1)
    q = rand_cloud(5000, 2, scale=11)
    ids, d2, tp, tn = ctx.knn(pts, q, k=k, eps=eps)
    oids, od2, otp, otn = oracle.Tree(pts).knn(q, k=k, eps=eps)
    np.testing.assert_array_equal(ids, oids)
    np.testing.assert_array_equal(d2, od2)
    assert tp == otp and tn == otn


def test_knn_scene_and_duplicates(ctx, oracle):
    pr = sy.make_pair(30000, 10000, seed=4)
    pts = pr.ref.copy()
    pts[1000:1500] = pts[1000]  # duplicate block
    ids, d2, tp, tn = ctx.knn(pts, pr.read, k=1, eps=3.16)
    oids, od2, otp, otn = oracle.Tree(pts).knn(pr.read, k=1, eps=3.16)
    np.testing.assert_array_equal(ids, oids)
    np.testing.assert_array_equal(d2, od2)
    assert tp == otp


def test_knn_max_radius_and_tiny(ctx, oracle):
    pts = rand_cloud(3, 5)
    q = rand_cloud(100, 6)
    ids, d2, _, _ = ctx.knn(pts, q, k=1, eps=0.0, max_dist=5.0)
    oids, od2, _, _ = oracle.Tree(pts).knn(q, k=1, eps=0.0, max_radius=5.0)
    np.testing.assert_array_equal(ids, oids)
    np.testing.assert_array_equal(d2, od2)
    ids, d2, _, _ = ctx.knn(pts[:1], q, k=4)  # fewer points than k
    oids, od2, _, _ = oracle.Tree(pts[:1]).knn(q, k=4)
    np.testing.assert_array_equal(ids, oids)
    np.testing.assert_array_equal(d2, od2)


# ---------------------------------------------------------------- normals -----------------
def test_normals_match_oracle(ctx, oracle):
    P = sy.make_pair(15000, 10, seed=3).ref
    n_gpu, deg_gpu = ctx.normals(P, knn=20)
    n_cpu, _, deg_cpu = oracle.surface_normals(P, knn=20)
    assert deg_gpu == deg_cpu
    dots = np.abs(np.sum(n_gpu.astype(np.float64) * n_cpu, 1))
    assert np.all(dots > 1 - 1e-6), dots.min()
    assert np.mean(np.all(n_gpu == n_cpu, axis=1)) > 0.99  # same tree, same neighbours, same solver


@pytest.mark.parametrize("engine", [1, 2])
def test_normals_knn_engines_identical(ctx, oracle, engine):
    """The SurfaceNormal kNN engines (one query per octet of lanes, k_knn_oct; one per lane,
    k_knn_ids) keep libnabo's visit order and replaceHead semantics, ties included: on a scene
    with a block of duplicate points their normals are bit-identical to each other and to the
    oracle's."""
    P = sy.make_pair(15000, 10, seed=3).ref.copy()
    P[2000:2040] = P[2000]  # 40 duplicates: exact distance ties in the k-best lists
    with ctx.options(normals_knn_engine=engine):
        n_gpu, deg_gpu = ctx.normals(P, knn=20)
    with ctx.options(normals_knn_engine=2):
        n_lane, deg_lane = ctx.normals(P, knn=20)
    assert deg_gpu == deg_lane
    np.testing.assert_array_equal(n_gpu, n_lane)
    n_cpu, _, deg_cpu = oracle.surface_normals(P, knn=20)
    assert deg_gpu == deg_cpu
    assert np.mean(np.all(n_gpu == n_cpu, axis=1)) > 0.99


def test_normals_degenerate(ctx, oracle):
    x = np.linspace(0, 5, 300, dtype=np.float32)
    P = np.c_[x, np.zeros_like(x), np.zeros_like(x)]
    n_gpu, deg = ctx.normals(P, knn=20)
    assert deg == 300
    np.testing.assert_array_equal(n_gpu, np.tile([0, 1, 0], (300, 1)).astype(np.float32))


# ---------------------------------------------------------------- trimmed quantile --------
@pytest.mark.parametrize("n", [1, 7, 1000, 131071, 500000])
@pytest.mark.parametrize("q", [0.25, 0.358818, 0.5, 0.7, 1.0])
def test_quantile_exact(ctx, oracle, n, q):
    rng = np.random.default_rng(n)
    d2 = rng.exponential(size=n).astype(np.float32) ** 3
    if n > 10:
        d2[::13] = np.inf
        d2[3 : n // 3] = d2[2]  # heavy ties
    ref, err = oracle.dists_quantile(d2, q)
    assert err == 0
    assert ctx.dists_quantile(d2, q) == ref


def test_quantile_no_outlier_to_filter(ctx, L):
    with pytest.raises(L.ConvergenceError):
        ctx.dists_quantile(np.full(100, np.inf, np.float32), 0.5)


# ---------------------------------------------------------------- 6x6 solve ---------------
@pytest.mark.parametrize("rank", [6, 5, 3, 1])
def test_solve6_matches_oracle(ctx, oracle, rank):
    rng = np.random.default_rng(20 + rank)
    F = rng.normal(size=(6, rank)) @ rng.normal(size=(rank, 400))
    A = F @ F.T
    b = F @ rng.normal(size=400)
    x, path = ctx.solve6(A, b)
    xo, po_ = oracle.solve6(A, b)
    assert path == po_
    np.testing.assert_allclose(x, xo, rtol=1e-9, atol=1e-12)


# ---------------------------------------------------------------- overlap -----------------
@pytest.mark.parametrize("seed,half", [(1, 10.0), (2, 30.0)])
def test_overlap_counts_exact(ctx, oracle, L, seed, half):
    pr = sy.make_pair(20000, 18000, seed=seed, half=half)
    _, st, rc = ctx.align_batch([dict(ref=pr.ref, read=pr.read, ref_origin=pr.ref_origin,
                                      read_origin=pr.read_origin)], flags=L.AICP_RUN_OVERLAP, resolution=RES)
    ov, cnt = oracle.overlap(pr.ref, pr.ref_origin, pr.read, pr.read_origin, RES)
    assert st[0]["overlap_keys"] == [int(c) for c in cnt]
    assert st[0]["overlap_percent"] == np.float32(ov)


def test_overlap_identical_clouds_is_100(ctx, L):
    pr = sy.make_pair(5000, 10, seed=3)
    _, st, _ = ctx.align_batch([dict(ref=pr.ref, read=pr.ref, ref_origin=pr.ref_origin,
                                     read_origin=pr.ref_origin)], flags=L.AICP_RUN_OVERLAP, resolution=RES)
    assert st[0]["overlap_percent"] == 100.0


def test_overlap_far_outlier(ctx, oracle, L):
    """One return 300 m away (a long ray, a wide key box): counts still equal the oracle's."""
    pr = sy.make_pair(6000, 6000, seed=31)
    read = np.vstack([pr.read, [[300.0, 2.0, 1.0]]]).astype(np.float32)
    _, st, rc = ctx.align_batch([dict(ref=pr.ref, read=read, ref_origin=pr.ref_origin,
                                      read_origin=pr.read_origin)], flags=L.AICP_RUN_OVERLAP, resolution=RES)
    ov, cnt = oracle.overlap(pr.ref, pr.ref_origin, read, pr.read_origin, RES)
    assert rc == 0
    assert st[0]["overlap_keys"] == [int(c) for c in cnt]


def test_overlap_extreme_outlier_sparse_path(ctx, oracle, L):
    """A return kilometres away in every axis makes a key box of ~10^13 voxels: the batch takes the
    sorted-key path (kernels_overlap_sparse.hip) and the key counts still equal the oracle's, like
    octomap, whose sparse tree accepts any in-range key (octrees_overlap.cpp:184)."""
    pr = sy.make_pair(3000, 3000, seed=32)
    read = np.vstack([pr.read, [[5000.0, 5000.0, 5000.0]]]).astype(np.float32)
    _, st, rc = ctx.align_batch([dict(ref=pr.ref, read=read, ref_origin=pr.ref_origin,
                                      read_origin=pr.read_origin)], flags=L.AICP_RUN_OVERLAP, resolution=RES)
    ov, cnt = oracle.overlap(pr.ref, pr.ref_origin, read, pr.read_origin, RES)
    assert rc == 0
    assert st[0]["overlap_keys"] == [int(c) for c in cnt]
    assert st[0]["overlap_percent"] == np.float32(ov)


def test_overlap_sparse_path_equals_dense(ctx, oracle, L):
    """The option overlap_path = 1 forces the sorted-key path on an ordinary ragged batch with a shared
    reference: every pair's three counts and ratio equal the voxel-map path's and the oracle's."""
    seq = sy.make_sequence(n_readings=4, ref_every=2, n_points=6000, seed=5, half=20.0)
    pairs = [dict(ref=p.ref, read=p.read[: 4000 + 500 * i], ref_origin=p.ref_origin, read_origin=p.read_origin)
             for i, p in enumerate(seq)]
    T0, s0, rc0 = ctx.align_batch(pairs, flags=L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP, resolution=RES)
    with ctx.options(overlap_path=1):
        T1, s1, rc1 = ctx.align_batch(pairs, flags=L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP, resolution=RES)
    assert rc0 == rc1 == 0
    np.testing.assert_array_equal(T0, T1)
    for a, b, p in zip(s0, s1, pairs):
        assert a["overlap_keys"] == b["overlap_keys"] and a["trimmed_ratio"] == b["trimmed_ratio"]
        ov, cnt = oracle.overlap(p["ref"], p["ref_origin"], p["read"], p["read_origin"], RES)
        assert b["overlap_keys"] == [int(c) for c in cnt]


# ---------------------------------------------------------------- whole ICP ---------------
def _icp_case(ctx, oracle, pr, ratio, eps=3.16, T0=None):
    cfg = ctx_cfg = None
    import aicp_mapping_amd._lib as L

    ctx_cfg = L.default_config(trimmed_ratio=ratio, nn_epsilon=eps)
    T, st, rc = ctx.align_batch([dict(ref=pr.ref, read=pr.read, init_T=T0)], ctx_cfg, flags=L.AICP_RUN_ICP)
    # reference semantics: SurfaceNormal on the raw reference, then centring
    ocfg = oracle.default_config(trimmed_ratio=ratio, nn_epsilon=eps, normals_on_centered=0)
    rc1, T1, st1 = oracle.icp(pr.ref, pr.read, ocfg, T0=T0)
    return T[0], st[0], (rc1, T1, st1), (rc1, T1, st1)


@pytest.mark.parametrize("seed,n,ratio", [(1, 20000, 0.6), (5, 8000, 0.358818), (9, 30000, 0.7)])
def test_icp_matches_oracle(ctx, oracle, seed, n, ratio):
    pr = sy.make_pair(n, n, seed=seed)
    T, st, (rc1, T1, st1), (rc0, T0r, st0) = _icp_case(ctx, oracle, pr, ratio)
    assert st["status"] == 0 and rc1 == 0 and rc0 == 0
    r, t = sy.rot_err(T1, T)  # same normal layout: near bit-exact
    assert r < 1e-6 and t < 1e-5, (r, t)
    assert st["iterations"] == st1.iterations
    r0, t0 = sy.rot_err(T0r, T)  # reference semantics (normals on raw coordinates)
    assert r0 <= ROT_TOL and t0 <= TRANS_TOL, (r0, t0)
    rg, tg = sy.rot_err(pr.T_gt, T)
    assert rg < 2e-3 and tg < 2e-2


@pytest.mark.parametrize("bucket,force", [(16, 0), (8, 1), (3, 0)])
def test_node_record_engine_matches_oracle(ctx, oracle, L, bucket, force):
    """The NN engine over node records (Trav<1>) serves chains with KDTreeMatcher bucketSize
    above 15 (treelet leaf slots hold 4-bit counts), references above 4 M points and batches
    past 2^28 treelet records; the option nn_engine = 1 selects it on a normal cloud. Both paths give
    the oracle's transform, iteration count and libnabo touch counts; SurfaceNormal keeps its own
    bucket-8 tree whatever the matcher's bucketSize."""
    pr = sy.make_pair(20000, 20000, seed=61)
    cfg = L.default_config(trimmed_ratio=0.6, bucket_size=bucket)
    with ctx.options(nn_engine=force):
        T, st, rc = ctx.align_batch([dict(ref=pr.ref, read=pr.read)], cfg, flags=L.AICP_RUN_ICP)
    rc1, T1, st1 = oracle.icp(pr.ref, pr.read, oracle.default_config(trimmed_ratio=0.6, bucket_size=bucket))
    assert rc == 0 and rc1 == 0
    r, t = sy.rot_err(T1, T[0])
    assert r < 1e-6 and t < 1e-5, (r, t)
    assert st[0]["iterations"] == st1.iterations
    assert (st[0]["nn_points_touched"], st[0]["nn_nodes_touched"]) == (st1.nn_points_touched, st1.nn_nodes_touched)
    assert st[0]["degenerate_normals"] == st1.degenerate_normals


def test_transformation_error_non_rigid_init(ctx, oracle, L):
    """A non-rigid initial transform: ICP::compute applies T_refMean_dataIn to the reading and
    RigidTransformation::checkParameters throws TransformationError (|1 - det R| > 0.001); the
    device reports AICP_ERR_TRANSFORMATION like the oracle's status 5, and the context keeps
    working."""
    pr = sy.make_pair(5000, 5000, seed=62)
    T0 = np.eye(4)
    T0[:3, :3] *= 1.01  # det 1.0303
    _, st, rc = ctx.align_batch([dict(ref=pr.ref, read=pr.read, init_T=T0)], L.default_config(trimmed_ratio=0.6),
                                flags=L.AICP_RUN_ICP, raise_on_error=False)
    rc1, _, _ = oracle.icp(pr.ref, pr.read, oracle.default_config(trimmed_ratio=0.6), T0=T0)
    assert rc == L.AICP_ERR_TRANSFORMATION and st[0]["status"] == L.AICP_ERR_TRANSFORMATION and rc1 == 5
    with pytest.raises(L.TransformationError):
        ctx.align_batch([dict(ref=pr.ref, read=pr.read, init_T=T0)], L.default_config(trimmed_ratio=0.6),
                        flags=L.AICP_RUN_ICP)
    T0[:3, :3] = np.eye(3) * 0.99985  # det 0.99955: within the 0.001 tolerance, accepted
    _, st, rc = ctx.align_batch([dict(ref=pr.ref, read=pr.read, init_T=T0)], L.default_config(trimmed_ratio=0.6),
                                flags=L.AICP_RUN_ICP, raise_on_error=False)
    rc1, _, _ = oracle.icp(pr.ref, pr.read, oracle.default_config(trimmed_ratio=0.6), T0=T0)
    assert rc == 0 and rc1 == 0


def test_icp_initial_transform(ctx, oracle):
    pr = sy.make_pair(10000, 10000, seed=11)
    T0 = sy.make_T(yaw_deg=1.5, pitch_deg=0.0, roll_deg=0.0, t=(0.1, -0.05, 0.0))
    T, st, (rc1, T1, st1), _ = _icp_case(ctx, oracle, pr, 0.6, T0=T0)
    r, t = sy.rot_err(T1, T)
    assert r < 1e-6 and t < 1e-5


def test_icp_cube_validation_recipe(ctx, oracle):
    # bash/run_registration_validation.sh + registration_main.cpp:331-347 perturbation
    cube = sy.make_cube()
    rng = np.random.default_rng(3)
    for _ in range(3):
        T = sy.make_T(yaw_deg=rng.normal(0, 1.0), pitch_deg=0, roll_deg=0,
                      t=(rng.normal(0, 0.1), rng.normal(0, 0.1), 0.0))
        read = sy.transform(np.linalg.inv(T), cube)
        pr = sy.Pair(cube, read, np.zeros(3), np.zeros(3), T)
        Tg, st, (rc1, T1, st1), (rc0, T0r, _) = _icp_case(ctx, oracle, pr, 0.7)
        r, t = sy.rot_err(T1, Tg)
        assert r < 1e-6 and t < 1e-5
        r0, t0 = sy.rot_err(T0r, Tg)
        assert r0 <= ROT_TOL and t0 <= TRANS_TOL


def test_icp_planar_rank_deficient(ctx, oracle):
    x = np.linspace(-5, 5, 400)
    P = np.c_[np.r_[x, x, np.full(400, -5.0)], np.r_[np.full(400, -3.0), np.full(400, 3.0), x * 0.6],
              np.zeros(1200)].astype(np.float32)
    rng = np.random.default_rng(0)
    P[:, :2] += rng.normal(0, 0.01, (1200, 2)).astype(np.float32)
    T = sy.make_T(yaw_deg=1.0, pitch_deg=0, roll_deg=0, t=(0.05, 0.03, 0))
    pr = sy.Pair(P, sy.transform(np.linalg.inv(T), P), np.zeros(3), np.zeros(3), T)
    Tg, st, (rc1, T1, st1), _ = _icp_case(ctx, oracle, pr, 0.7)
    assert st["status"] == rc1 == 0
    r, t = sy.rot_err(T1, Tg)
    assert r < 1e-6 and t < 1e-5


def test_icp_convergence_error(ctx, L):
    pr = sy.make_pair(3000, 3000, seed=2)
    cfg = L.default_config(trimmed_ratio=0.5, nn_max_dist=1e-6)
    _, st, rc = ctx.align_batch([dict(ref=pr.ref, read=pr.read + 5.0)], cfg, raise_on_error=False)
    assert rc == L.AICP_ERR_CONVERGENCE and st[0]["status"] == L.AICP_ERR_CONVERGENCE


# ---------------------------------------------------------------- pipeline + batches ------
def test_align_batch_ragged_matches_oracle(ctx, oracle, L):
    sizes = [(6000, 5000), (12000, 15000), (3000, 3500), (9000, 9000)]
    pairs, prs = [], []
    for i, (m, n) in enumerate(sizes):
        pr = sy.make_pair(m, n, seed=30 + i, half=20.0)
        prs.append(pr)
        pairs.append(dict(ref=pr.ref, read=pr.read, ref_origin=pr.ref_origin, read_origin=pr.read_origin))
    T, st, rc = ctx.align_batch(pairs, flags=L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP, resolution=RES)
    for i, pr in enumerate(prs):
        ov, cnt = oracle.overlap(pr.ref, pr.ref_origin, pr.read, pr.read_origin, RES)
        assert st[i]["overlap_keys"] == [int(c) for c in cnt]
        ratio = oracle.autotune_ratio(ov)
        assert st[i]["trimmed_ratio"] == np.float32(ratio)
        rc1, T1, st1 = oracle.icp(pr.ref, pr.read, oracle.default_config(trimmed_ratio=ratio, normals_on_centered=0))
        r, t = sy.rot_err(T1, T[i])
        assert r < 1e-6 and t < 1e-5, (i, r, t)
        assert st[i]["iterations"] == st1.iterations


def test_shared_reference_window(ctx, oracle, L):
    """C2 reference windows: pairs that pass the SAME reference array share one centroid,
    kd-tree and normals on the device; every pair must still match the oracle (which rebuilds
    them per registration, as libpointmatcher does), and match a batch with copied refs."""
    seq = sy.make_sequence(n_readings=6, ref_every=3, n_points=6000, seed=3, half=20.0)
    assert seq[0].ref is seq[2].ref and seq[3].ref is not seq[2].ref
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
    shared = [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in seq]
    copied = [dict(ref=p.ref.copy(), read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in seq]
    Ts, ss, _ = ctx.align_batch(shared, flags=flags, resolution=RES)
    Tc, sc, _ = ctx.align_batch(copied, flags=flags, resolution=RES)
    np.testing.assert_array_equal(Ts, Tc)
    assert [x["iterations"] for x in ss] == [x["iterations"] for x in sc]
    assert [x["degenerate_normals"] for x in ss] == [x["degenerate_normals"] for x in sc]
    for i, pr in enumerate(seq):
        ov, cnt = oracle.overlap(pr.ref, pr.ref_origin, pr.read, pr.read_origin, RES)
        assert ss[i]["overlap_keys"] == [int(c) for c in cnt]
        ratio = oracle.autotune_ratio(ov)
        rc1, T1, st1 = oracle.icp(pr.ref, pr.read, oracle.default_config(trimmed_ratio=ratio, normals_on_centered=0))
        r, t = sy.rot_err(T1, Ts[i])
        assert rc1 == 0 and r < 1e-6 and t < 1e-5, (i, r, t)
        assert ss[i]["iterations"] == st1.iterations


def test_batch_deterministic_and_order_independent(ctx, L):
    prs = [sy.make_pair(8000, 8000, seed=50 + i) for i in range(3)]
    pairs = [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs]
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
    Ta, sa, _ = ctx.align_batch(pairs, flags=flags, resolution=RES)
    Tb, sb, _ = ctx.align_batch(pairs[::-1], flags=flags, resolution=RES)
    Tc, sc, _ = ctx.align_batch(pairs[1:2], flags=flags, resolution=RES)
    np.testing.assert_array_equal(Ta, Tb[::-1])
    np.testing.assert_array_equal(Ta[1], Tc[0])


def test_select_one_workgroup_per_pair_equals_chip_wide(ctx, L):
    """k_sel_pair (the whole TrimmedDist select of a pair in one workgroup; batches of >= 256 pairs
    take it) gives the chip-wide select's limits: same transforms and statistics bit for bit, on
    ordinary pairs and on one whose distances all fall into one digit-1 bin (more candidates than
    the kernel keeps in LDS: its global-memory path). raw_tree_first's order (batches of >= 4 M
    reference points) changes nothing either."""
    prs = [sy.make_pair(9000 + 1500 * i, 12000 - 1000 * i, seed=70 + i) for i in range(4)]
    pairs = [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs]
    g = np.random.default_rng(7)
    plane = np.zeros((20000, 3), np.float32)
    plane[:, :2] = g.uniform(-10, 10, (20000, 2)).astype(np.float32)
    lifted = plane.copy()
    lifted[:, 2] = np.float32(0.1)  # every nearest distance^2 is 0.01: one bin, 20000 candidates
    pairs.append(dict(ref=plane, read=lifted, ref_origin=np.zeros(3), read_origin=np.zeros(3)))
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
    out = {}
    # also the batch path's stream order for large batches (the raw tree first, the matcher tree
    # from the raw tree's global levels on), forced on this small batch: same results
    for v, raw in ((0, 0), (1, 0), (0, 1), (1, 1)):
        with ctx.options(select_pair=v, raw_tree_first=raw):
            out[f"{v}{raw}"] = ctx.align_batch(pairs, flags=flags, resolution=RES)
    T0, s0, rc0 = out["00"]
    for k in ("10", "01", "11"):
        T1, s1, rc1 = out[k]
        assert rc0 == rc1, k
        np.testing.assert_array_equal(T0, T1)
        assert s0 == s1, k


def test_concurrent_contexts_identical(ctx, L):
    """Two contexts on one device driven by two host threads at once (bench.py --lanes): each
    batch's transforms and touch counts equal a lone run's (no shared device state)."""
    import threading

    prs = [sy.make_pair(20000, 20000, seed=90 + i) for i in range(4)]
    pairs = [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs]
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
    T0, s0, rc0 = ctx.align_batch(pairs, flags=flags, resolution=RES)
    assert rc0 == 0
    ctxs = [L.Context(0), L.Context(0)]
    batches = [c.upload(pairs) for c in ctxs]
    out = [None, None]

    def work(i):
        for _ in range(3):
            batches[i].run(L.default_config(), RES, flags)
        out[i] = (batches[i].transforms(), batches[i].stats_dicts())

    th = [threading.Thread(target=work, args=(i,)) for i in range(2)]
    for t in th:
        t.start()
    for t in th:
        t.join()
    for T, st in out:
        np.testing.assert_array_equal(T, T0)
        for a, b in zip(st, s0):
            assert (a["iterations"], a["nn_points_touched"], a["nn_nodes_touched"]) == \
                   (b["iterations"], b["nn_points_touched"], b["nn_nodes_touched"])
    for b in batches:
        b.free()
    for c in ctxs:
        c.close()


@pytest.mark.parametrize("plan", [1, 2, -1])
def test_planned_tree_build(ctx, L, plan):
    """The kd-trees are built with a planned number of global levels and no host read-back.
    A plan too shallow for the data (1 or 2 levels here) leaves segments above the wave-LDS
    size, which the subtree kernel finishes in global memory; -1 is the host-polled build.
    Every variant must give the default build's transforms, depths and touch counts."""
    prs = [sy.make_pair(30000, 30000, seed=70 + i) for i in range(2)]
    pairs = [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs]
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
    Ta, sa, rca = ctx.align_batch(pairs, flags=flags, resolution=RES)
    with ctx.options(tree_plan=plan):
        Tb, sb, rcb = ctx.align_batch(pairs, flags=flags, resolution=RES)
    assert rca == rcb == 0
    np.testing.assert_array_equal(Ta, Tb)
    for a, b in zip(sa, sb):
        assert (a["iterations"], a["tree_depth"], a["nn_points_touched"], a["nn_nodes_touched"]) == \
               (b["iterations"], b["tree_depth"], b["nn_points_touched"], b["nn_nodes_touched"])


def test_tree_scan_stall_fails_safely(ctx, L):
    """A kd-tree scan whose look-back gives up (kernels_tree.hip lookback_scan; never seen, the
    pattern that cost r05 a box when a grid barrier timed out) recomputes its exact prefix, so no
    later kernel indexes with a partial one, and reports error 16: forced through the test hook on
    every tile but the first, the call returns AICP_ERR_HIP without a fault, and the context's next
    call gives the results of the run before."""
    prs = [sy.make_pair(30000, 30000, seed=40 + i) for i in range(2)]  # two references: no cache
    pairs = [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs]
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
    T0, s0, rc0 = ctx.align_batch(pairs, flags=flags, resolution=RES)
    assert rc0 == 0
    assert L.test_force_scan_stall(True) == L.AICP_OK
    try:
        _, _, rc1 = ctx.align_batch(pairs, flags=flags, resolution=RES, raise_on_error=False)
    finally:
        assert L.test_force_scan_stall(False) == L.AICP_OK
    assert rc1 == L.AICP_ERR_HIP and "16" in ctx.last_error(), (rc1, ctx.last_error())
    T2, s2, rc2 = ctx.align_batch(pairs, flags=flags, resolution=RES)
    assert rc2 == 0
    np.testing.assert_array_equal(T0, T2)
    assert s0 == s2


def test_block_subtree_builder_matches_oracle_trees(ctx, oracle, L):
    """k_tr_subtree_blk (the waves of a block take the nodes of a level) builds libnabo's trees:
    the touch counts depend on every node of the matcher tree and the normals on the raw tree."""
    prs = [sy.make_pair(25000, 25000, seed=80 + i) for i in range(2)]
    pairs = [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs]
    T, st, rc = ctx.align_batch(pairs, flags=L.AICP_RUN_ICP, cfg=L.default_config(trimmed_ratio=0.65))
    assert rc == 0
    for i, p in enumerate(prs):
        rc1, T1, st1 = oracle.icp(p.ref, p.read, oracle.default_config(trimmed_ratio=0.65))
        assert (st[i]["nn_points_touched"], st[i]["nn_nodes_touched"], st[i]["tree_depth"]) == \
               (st1.nn_points_touched, st1.nn_nodes_touched, st1.tree_depth)
        assert st[i]["degenerate_normals"] == st1.degenerate_normals
        r, t = sy.rot_err(T1, T[i])
        assert r < 1e-6 and t < 1e-5


@pytest.mark.parametrize("builder", ["level", "block", "block_b6"])
def test_subtree_builders_match_oracle_trees(ctx, oracle, L, builder):
    """The finishing builders below the global levels give libnabo's trees (touch counts, depth,
    normals): k_tr_subtree_lvl (all nodes of a level per pass; builds of >= 4 M points, forced
    here), k_tr_subtree_blk (a node per wave) with bucketSize 8 and 6."""
    bucket = 6 if builder == "block_b6" else 8
    prs = [sy.make_pair(20000, 20000, seed=90 + i) for i in range(2)]
    pairs = [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs]
    with ctx.options(tree_lvl_min=1 if builder == "level" else L.default_options().tree_lvl_min):
        T, st, rc = ctx.align_batch(pairs, flags=L.AICP_RUN_ICP,
                                    cfg=L.default_config(trimmed_ratio=0.65, bucket_size=bucket))
    assert rc == 0
    for i, p in enumerate(prs):
        rc1, T1, st1 = oracle.icp(p.ref, p.read, oracle.default_config(trimmed_ratio=0.65, bucket_size=bucket))
        assert (st[i]["nn_points_touched"], st[i]["nn_nodes_touched"], st[i]["tree_depth"]) == \
               (st1.nn_points_touched, st1.nn_nodes_touched, st1.tree_depth)
        assert st[i]["degenerate_normals"] == st1.degenerate_normals
        r, t = sy.rot_err(T1, T[i])
        assert r < 1e-6 and t < 1e-5


def test_resident_batch_full_size_round_trip(ctx, L):
    """C2 size (N = M = 120k): properties at full size (recovers T_gt, repeatable)."""
    prs = [sy.make_pair(120000, 120000, seed=100 + i) for i in range(2)]
    b = ctx.upload([dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs])
    b.run(resolution=RES)
    T1 = b.transforms()
    st = b.stats_dicts()
    b.run(resolution=RES)
    np.testing.assert_array_equal(T1, b.transforms())
    for i, p in enumerate(prs):
        r, t = sy.rot_err(p.T_gt, T1[i])
        assert r < 1e-3 and t < 1e-2, (r, t)
        assert 0.25 <= st[i]["trimmed_ratio"] <= 0.7 and 4 <= st[i]["iterations"] <= 20
    b.free()


def test_transform_matches_reference_float_order(ctx, oracle):
    P = rand_cloud(1000, 9)
    T = sy.make_T(yaw_deg=30, pitch_deg=5, roll_deg=-3, t=(1, 2, 3)).astype(np.float32)
    out = ctx.transform(T, P)
    exp = np.empty_like(P)
    for r in range(3):
        s = T[r, 0] * P[:, 0]
        s = (s + T[r, 1] * P[:, 1]).astype(np.float32)
        s = (s + T[r, 2] * P[:, 2]).astype(np.float32)
        exp[:, r] = (s + T[r, 3]).astype(np.float32)
    np.testing.assert_array_equal(out, exp)


def test_registration_interface_mirror(ctx, oracle, tmp_path):
    from aicp_mapping_amd import registration as R

    import shutil, os

    src = os.path.join(os.path.dirname(__file__), "golden", "icp_autotuned_default.yaml")
    reg = R.RegistrationParams(type="HIP")
    reg.pointmatcher.configFileName = src
    ovp = R.OverlapParams(type="OctreeBased")
    pipe = R.AicpPipeline(reg, ovp, registration_config_file=str(tmp_path / "icp_autotuned.yaml"), ctx=ctx)
    pr = sy.make_pair(8000, 8000, seed=77)
    Pr = np.eye(4); Pr[:3, 3] = pr.ref_origin
    Pd = np.eye(4); Pd[:3, 3] = pr.read_origin
    T = pipe.runAicpPipeline(pr.ref, pr.read, Pr, Pd)
    ov, _ = oracle.overlap(pr.ref, pr.ref_origin, pr.read, pr.read_origin, RES)
    assert pipe.octree_overlap_ == np.float32(ov)
    ratio = oracle.autotune_ratio(ov)
    assert ("ratio: %g" % ratio) in open(tmp_path / "icp_autotuned.yaml").read()
    rc1, T1, _ = oracle.icp(pr.ref, pr.read, oracle.default_config(trimmed_ratio=ratio, normals_on_centered=0))
    r, t = sy.rot_err(T1, T)
    assert r < 1e-6 and t < 1e-5
    out = pipe.registr_.getOutputReading()
    assert out.shape == (8000, 3)
    assert R.create_registrator(R.RegistrationParams(type="Nope")) is None


def test_pcl_point_layouts_register_identically(ctx):
    """registerClouds over PointXYZ / PointXYZRGB / PointXYZRGBNormal rows (stride 16 / 32 / 48 B,
    abstract_registrator.hpp:10-12): the strided loads give the packed-xyz transform bit for bit."""
    pr = sy.make_pair(6000, 6000, seed=23)
    base = None
    for w in (3, 4, 8, 12):
        ref = np.full((len(pr.ref), w), 7.0, np.float32)
        read = np.full((len(pr.read), w), -3.0, np.float32)
        ref[:, :3], read[:, :3] = pr.ref, pr.read
        T, st, rc = ctx.align_batch([dict(ref=ref, read=read, ref_origin=pr.ref_origin,
                                          read_origin=pr.read_origin)],
                                    flags=ctx_flags_all())
        assert rc == 0
        if base is None:
            base = T
        assert np.array_equal(T, base)


def ctx_flags_all():
    import aicp_mapping_amd._lib as L

    return L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
