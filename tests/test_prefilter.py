"""Pre-filter regionGrowingUniformPlaneSegmentationFilter (filteringUtils.cpp:5-103), SURVEY §8(f)
rank 2: the oracle's restatement (oracle/prefilter_oracle.cpp) and the device path
(kernels_prefilter.hip) through the C-ABI.

PARITY UNPINNED: PCL is absent here and the reference holds no fixture for this path. The
oracle is checked against independent numpy computations (voxel centroids, normals from
numpy's eigh, and the min-label formulation of region growing that the device uses) and the
device against the oracle. Bar: bit-exact sampled points, normals, curvatures, cluster labels
and output (integer/index work and the same float expressions in the same order); the only
transcendental functions (atan2/cos/sin of computeRoots) run in double on both sides and are
rounded to float.
"""
import numpy as np
import pytest

from aicp_mapping_amd import synthetic as sy


def scene_cloud(seed=3, half=6.0, spacing=0.04, origin=(0.0, 0.0, 0.7)):
    sc = sy.make_scene(seed)
    rng = np.random.default_rng(seed + 100)
    return sy.sample_scene(sc, rng, origin, half=half, spacing=spacing).astype(np.float32)


def voxel_numpy(P, leaf=0.08):
    """VoxelGrid by numpy: float32 keys like PCL, stable grouping, float32 sums in input order."""
    P = P[np.isfinite(P).all(1)]
    inv = np.float32(1.0) / np.float32(leaf)
    lo, hi = P.min(0), P.max(0)
    minb = np.floor(lo * inv).astype(np.int64)
    div = np.floor(hi * inv).astype(np.int64) - minb + 1
    ijk = (np.floor(P * inv) - minb.astype(np.float32)).astype(np.int64)
    key = ijk[:, 0] + ijk[:, 1] * div[0] + ijk[:, 2] * div[0] * div[1]
    order = np.argsort(key, kind="stable")
    ks = key[order]
    heads = np.r_[True, ks[1:] != ks[:-1]]
    starts = np.nonzero(heads)[0]
    ends = np.r_[starts[1:], len(ks)]
    out = np.empty((len(starts), 3), np.float32)
    for v, (b, e) in enumerate(zip(starts, ends)):
        c = P[order[b]].copy()
        for i in range(b + 1, e):
            c = (c + P[order[i]]).astype(np.float32)
        out[v] = c / np.float32(e - b)
    return out


def min_label_regions(sampled, nbr, cos_thr, curv_thr, min_size=50, max_size=1000000):
    """The device formulation (kernels_prefilter.hip): label = min seed-order position over
    prop points reaching the point, then non-prop seeds grown one level in order."""
    V = len(sampled)
    N, curv = sampled[:, 4:7], sampled[:, 3]
    nb = nbr[:, :]
    valid = np.zeros(nb.shape, bool)
    for t in range(nb.shape[1]):
        y = nb[:, t]
        ok = y >= 0
        d = np.abs(N[y, 0] * N[:, 0] + (N[y, 1] * N[:, 1] + N[y, 2] * N[:, 2]))
        valid[:, t] = ok & ~(d < cos_thr)
    prop = ~(curv > curv_thr)
    key = np.where(np.isnan(curv), np.inf, curv)
    order = np.lexsort((np.arange(V), np.isnan(curv), key))
    order_of = np.empty(V, np.int64)
    order_of[order] = np.arange(V)
    INF = np.iinfo(np.int64).max
    lab = np.where(prop, order_of, INF)
    src = np.repeat(np.arange(V), nb.shape[1])[valid.ravel()]
    dst = nb.ravel()[valid.ravel()]
    keep = prop[src]
    src, dst = src[keep], dst[keep]
    while True:
        old = lab.copy()
        f = lab < INF
        lab[f] = np.minimum(lab[f], lab[order[lab[f]]])
        np.minimum.at(lab, dst, lab[src])
        if (lab == old).all():
            break
    for q in range(V):
        x = order[q]
        if lab[x] != INF:
            continue
        lab[x] = q
        for t in range(nb.shape[1]):
            y = nb[x, t]
            if y < 0:
                break
            if valid[x, t] and lab[y] == INF:
                lab[y] = q
    uniq, cnt = np.unique(lab, return_counts=True)
    kept = uniq[(cnt >= min_size) & (cnt <= max_size)]
    cid = {int(u): i for i, u in enumerate(kept)}
    return np.array([cid.get(int(v), -1) for v in lab], np.int32)


def sorted_knn(oracle, P, k):
    t = oracle.Tree(P)
    ids, d2 = t.knn(P, k=k)[:2]
    out = np.empty_like(ids)
    for i in range(len(P)):
        out[i] = [b for _, b in sorted(zip(d2[i].tolist(), ids[i].tolist()), key=lambda x: (x[0], x[1]))]
    return out


# ------------------------------------------------------------------- oracle (CPU) ----------
def test_oracle_voxel_grid_matches_numpy(oracle):
    P = scene_cloud(half=3.0)
    r = oracle.prefilter(P)
    ref = voxel_numpy(P)
    assert r["sampled"].shape[0] == len(ref)
    assert np.array_equal(r["sampled"][:, :3], ref)


def test_oracle_normals_match_numpy_eigh(oracle):
    P = scene_cloud(half=3.0)
    r = oracle.prefilter(P)
    s = r["sampled"]
    nb = sorted_knn(oracle, s[:, :3].copy(), 30)
    rng = np.random.default_rng(0)
    for i in rng.choice(len(s), 300, replace=False):
        Q = s[nb[i], :3].astype(np.float64)
        C = np.cov(Q.T, bias=True)
        w, U = np.linalg.eigh(C)
        n = U[:, 0]
        if w[1] < 50 * max(w[0], 1e-12):  # skip ill-conditioned neighbourhoods (edges, corners)
            continue
        assert abs(abs(float(n @ s[i, 4:7])) - 1.0) < 1e-3
        assert abs(w[0] / w.sum() - s[i, 3]) < 2e-3
        assert float(s[i, 4:7] @ (0 - s[i, :3])) >= 0  # flipped towards the viewpoint (origin)


@pytest.mark.parametrize("curv_thr", [1.0, 0.02])
def test_oracle_region_growing_equals_min_label_formulation(oracle, curv_thr):
    P = scene_cloud(seed=5, half=7.0)
    prm = oracle.prefilter_params(curvature=curv_thr)
    r = oracle.prefilter(P, prm)
    s = r["sampled"]
    nb = sorted_knn(oracle, s[:, :3].copy(), 30)[:, :15]
    lab = min_label_regions(s, nb, prm.cos_smoothness, curv_thr)
    assert r["n_clusters"] > 3
    if curv_thr < 1.0:
        assert (s[:, 3] > curv_thr).sum() > 100  # the non-prop path is exercised
    assert np.array_equal(lab, r["labels"])
    # output = clusters in order, points ascending
    exp = np.concatenate([s[r["labels"] == c, :3] for c in range(r["n_clusters"])], 0)
    assert np.array_equal(exp, r["out"])


def test_oracle_edge_cases(oracle):
    e = oracle.prefilter(np.zeros((0, 3), np.float32))
    assert e["out"].shape == (0, 3) and e["sampled"].shape[0] == 0
    nan = np.full((10, 3), np.nan, np.float32)
    assert oracle.prefilter(nan)["sampled"].shape[0] == 0
    two = np.array([[0, 0, 0], [1, 1, 1]], np.float32)
    r = oracle.prefilter(two)
    assert r["sampled"].shape[0] == 2 and np.isnan(r["sampled"][:, 3]).all() and r["out"].shape[0] == 0
    few = np.random.default_rng(2).uniform(0, 1, size=(40, 3)).astype(np.float32)  # < min cluster size
    r = oracle.prefilter(few)
    assert 0 < r["sampled"].shape[0] < 50 and r["out"].shape[0] == 0


def test_oracle_overflow_passes_cloud_through(oracle):
    # extent / leaf beyond 32-bit voxel indices: PCL returns the input unfiltered
    rng = np.random.default_rng(1)
    P = rng.uniform(-1, 1, size=(400, 3)).astype(np.float32)
    P[0] = (-500, -500, -500)
    P[1] = (500, 500, 500)
    r = oracle.prefilter(P)
    assert np.array_equal(r["sampled"][:, :3], P)


# ------------------------------------------------------------------- device ----------------
@pytest.fixture(scope="module")
def ctx():
    import aicp_mapping_amd._lib as L

    c = L.Context(0)
    yield c
    c.close()


def _params(L, oracle, **kw):
    o = oracle.prefilter_params(**{k: v for k, v in kw.items() if k in ("curvature", "viewpoint", "neighbours",
                                                                         "normal_k")})
    d = L.default_prefilter()
    if "curvature" in kw:
        d.curvature_threshold = kw["curvature"]
    if "viewpoint" in kw:
        for i in range(3):
            d.viewpoint[i] = kw["viewpoint"][i]
    if "neighbours" in kw:
        d.neighbours = kw["neighbours"]
    if "normal_k" in kw:
        d.normal_k = kw["normal_k"]
    return d, o


def _check_same(g, r):
    assert g["sampled"].shape[0] == r["sampled"].shape[0]
    assert np.array_equal(g["sampled"][:, :3], r["sampled"][:, :3]), "voxel centroids"
    gs, rs = g["sampled"][:, 3:7], r["sampled"][:, 3:7]
    assert np.array_equal(np.isnan(gs), np.isnan(rs))
    m = ~np.isnan(rs)
    bad = np.nonzero((gs != rs) & m)[0]
    assert bad.size == 0, f"{bad.size} normals/curvatures differ, first {bad[:5]}: {gs[bad[:3]]} vs {rs[bad[:3]]}"
    assert g["n_clusters"] == r["n_clusters"]
    assert np.array_equal(g["labels"], r["labels"])
    assert np.array_equal(g["out"], r["out"])


@pytest.mark.gpu
def test_gpu_debug_order_transform_then_filter(ctx, oracle):
    """App's debug working mode moves the RAW reading by initialT_ and pre-filters the moved
    cloud (setAndFilterReading, app.cpp:87-99): AicpPipeline.setAndFilterReading does that on
    the device and equals the oracle's pcl::transformPointCloud followed by its pre-filter; the
    prior pose becomes fromMatrix4fToIsometry3d(initialT_) * pose."""
    from aicp_mapping_amd import registration as R
    from aicp_mapping_amd import synthetic as sy

    P = scene_cloud(seed=5, half=8.0)
    T = sy.make_T(yaw_deg=7.0, pitch_deg=1.0, roll_deg=-2.0, t=(0.4, -0.3, 0.05)).astype(np.float32)
    pose = sy.make_T(yaw_deg=3.0, pitch_deg=0.0, roll_deg=0.0, t=(1.0, 2.0, 0.7))
    pipe = R.AicpPipeline(R.RegistrationParams(type="HIP"), R.OverlapParams(type="OctreeBased"), ctx=ctx)
    got, gpose = pipe.setAndFilterReading(P, pose, "debug", T)
    want = oracle.prefilter(oracle.transform_cloud(T, P))["out"]
    assert np.array_equal(got, want)
    np.testing.assert_allclose(gpose[:3, 3], oracle.corrected_origin(T, pose[:3, 3]), rtol=0, atol=1e-12)
    robot, rpose = pipe.setAndFilterReading(P, pose)
    assert np.array_equal(robot, oracle.prefilter(P)["out"]) and np.array_equal(rpose, pose)


@pytest.mark.gpu
@pytest.mark.parametrize("seed,half", [(7, 5.0), (5, 8.0), (11, 12.0)])
def test_gpu_prefilter_matches_oracle(ctx, oracle, seed, half):
    import aicp_mapping_amd._lib as L

    P = scene_cloud(seed=seed, half=half)
    g = ctx.prefilter(P, details=True)
    r = oracle.prefilter(P)
    assert r["n_clusters"] > 3
    _check_same(g, r)


@pytest.mark.gpu
@pytest.mark.parametrize("curv", [0.02, 0.005])
def test_gpu_prefilter_non_prop_points(ctx, oracle, curv):
    """A low curvature threshold makes many points non-seeds (never queued) and leaves seeds
    for the sequential k_rg_phaseb."""
    import aicp_mapping_amd._lib as L

    P = scene_cloud(seed=7, half=5.0)
    d, o = _params(L, oracle, curvature=curv)
    g = ctx.prefilter(P, d, details=True)
    r = oracle.prefilter(P, o)
    assert (r["sampled"][:, 3] > curv).sum() > 100
    _check_same(g, r)


@pytest.mark.gpu
def test_gpu_prefilter_viewpoint_and_overload(ctx, oracle):
    from aicp_mapping_amd import filtering

    P = scene_cloud(seed=4, half=5.0)
    T = np.eye(4)
    T[:3, 3] = (3.0, -2.0, 5.0)
    clusters = []
    out = filtering.regionGrowingUniformPlaneSegmentationFilter(P, T, clusters, ctx=ctx)
    r = oracle.prefilter(P, oracle.prefilter_params(viewpoint=(3.0, -2.0, 5.0)))
    s = r["sampled"]
    assert out.shape == (len(s), 12)
    assert np.array_equal(out[:, :3], s[:, :3])
    assert np.array_equal(out[:, 4:7], s[:, 4:7]) and np.array_equal(out[:, 9], s[:, 3])
    assert len(clusters) == r["n_clusters"]
    for c, idx in enumerate(clusters):
        assert np.array_equal(idx, np.nonzero(r["labels"] == c)[0])
    kept = filtering.regionGrowingUniformPlaneSegmentationFilter(P, ctx=ctx)
    assert np.array_equal(kept, oracle.prefilter(P)["out"])
    prev = np.ones((5, 3), np.float32)
    acc = filtering.regionGrowingUniformPlaneSegmentationFilter(P, prev, ctx=ctx)
    assert np.array_equal(acc[:5], prev) and np.array_equal(acc[5:], kept)


@pytest.mark.gpu
@pytest.mark.parametrize("width", [4, 8, 12])
def test_gpu_prefilter_strided_layouts(ctx, oracle, width):
    P = scene_cloud(seed=6, half=3.0)
    W = np.zeros((len(P), width), np.float32)
    W[:, :3] = P
    W[:, 3:] = 7.0
    assert np.array_equal(ctx.prefilter(W), oracle.prefilter(P)["out"])


@pytest.mark.gpu
def test_gpu_prefilter_edge_cases(ctx, oracle):
    assert ctx.prefilter(np.zeros((0, 3), np.float32)).shape == (0, 3)
    nan = np.full((100, 3), np.nan, np.float32)
    g = ctx.prefilter(nan, details=True)
    assert g["sampled"].shape[0] == 0 and g["out"].shape[0] == 0
    for P in (np.array([[0, 0, 0], [1, 1, 1]], np.float32), scene_cloud(half=0.3)):
        _check_same(ctx.prefilter(P, details=True), oracle.prefilter(P))
    # non-finite points are skipped like PCL's !is_dense path
    P = scene_cloud(seed=9, half=3.0)
    Q = P.copy()
    Q[::7] = np.nan
    _check_same(ctx.prefilter(Q, details=True), oracle.prefilter(Q))
    # 32-bit voxel index overflow: the cloud passes unfiltered
    rng = np.random.default_rng(1)
    R = rng.uniform(-1, 1, size=(3000, 3)).astype(np.float32)
    R[0] = (-500, -500, -500)
    R[1] = (500, 500, 500)
    _check_same(ctx.prefilter(R, details=True), oracle.prefilter(R))


@pytest.mark.gpu
def test_gpu_prefilter_invalid_params(ctx):
    import aicp_mapping_amd._lib as L

    P = scene_cloud(half=2.0)
    with pytest.raises(L.AicpError):
        ctx.prefilter(P, L.default_prefilter(normal_k=25))
    with pytest.raises(L.AicpError):
        ctx.prefilter(P, L.default_prefilter(neighbours=17))
    with pytest.raises(L.AicpError):
        ctx.prefilter(P, L.default_prefilter(leaf_size=0.0))


@pytest.mark.gpu
def test_gpu_prefilter_map_scale(ctx, oracle):
    """A prior-map-sized input (app.cpp:491, app_ros.cpp:309): ~1.6 M points over 40 x 40 m."""
    P = scene_cloud(seed=2, half=20.0, spacing=0.035)
    assert len(P) > 1_000_000
    g = ctx.prefilter(P, details=True)
    r = oracle.prefilter(P)
    _check_same(g, r)
