"""CPU-side checks of the C-ABI library (no GPU needed): it loads, exports every symbol the
header declares, and its host-only entry points (chain parsing, ratio auto-tune, ratio
rewrite of the chain file) behave like the reference's host code. Plus the multi-rank
plumbing of bench.py on gloo with world_size 2.
"""
import ctypes as C
import math
import os
import re
import socket

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "aicp_hip.h")
GOLDEN = os.path.join(ROOT, "tests", "golden")


def header_functions():
    txt = open(HEADER).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    txt = re.sub(r"//[^\n]*", "", txt)
    return sorted(set(re.findall(r"\b(aicp_hip_[a-z0-9_]+)\s*\(", txt)))


@pytest.fixture(scope="module")
def L():
    import aicp_mapping_amd._lib as L

    return L


def test_library_exports_every_header_symbol(L):
    names = header_functions()
    assert len(names) >= 20
    so = C.CDLL(L.LIB_PATH)
    missing = [n for n in names if not hasattr(so, n)]
    assert not missing, missing
    assert sorted(L.EXPORTS) == names  # the Python mirror binds exactly the header


def test_library_is_gfx950_code_object(L):
    blob = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in blob
    assert b"k_icp_nn" in blob


def test_library_built_from_this_tree(L):
    """Provenance: the in-tree library's embedded source hash (aicp_hip_build_info, Makefile)
    equals the hash of the sources it sits next to, and it is a plain build (no diagnostic flags),
    so the binary that travels to the GPU box is the one these sources make."""
    info = L.build_info()
    assert info.startswith("src ") and " arch gfx950 " in info, info
    if os.environ.get("AICP_HIP_LIB"):
        pytest.skip("an A/B library override is loaded")
    p = L.provenance()
    assert p["built_from_tree"], p
    assert info.rstrip().endswith("extra"), info  # no -DAICP_DIAG / diagnostic flags


def test_version_and_defaults(L):
    assert L.lib.aicp_hip_version().decode().startswith("aicp_hip")
    c = L.default_config()
    # icp_autotuned_default.yaml:9-51 values
    assert (c.knn_normals, c.knn_match, c.max_iter, c.smooth_length, c.bucket_size) == (20, 1, 20, 4, 8)
    assert c.nn_epsilon == np.float32(3.16)
    assert c.trimmed_ratio == np.float32(0.70)
    assert c.min_diff_rot == np.float32(1e-3) and c.min_diff_trans == np.float32(1e-2)
    assert math.isinf(c.nn_max_dist)


def test_context_options_defaults_and_layout(L):
    """aicp_hip_options: the library's defaults are the product path, the ctypes mirror has the
    header's layout (14 32-bit fields, then a uint64), and nothing in the package reads the
    environment for them (r05 had 12 getenv switches in the library)."""
    import ctypes

    assert ctypes.sizeof(L.Options) == 64
    o = L.default_options().as_dict()
    assert o == dict(profile=0, nn_engine=0, overlap_path=0, normals_knn_engine=0, select_pair=-1,
                     select_fused_from=3, raw_tree_first=-1, raw_first_at=2, no_early_exit=0, tree_plan=0,
                     tree_lvl_min=1 << 22, reference_cache=1, oneshot_keep_mib=4096, early_reference=1,
                     read_order_min=200000)
    with pytest.raises(AttributeError):
        L.default_options(no_such_switch=1)
    src = "".join(open(os.path.join(ROOT, "aicp_mapping_amd", "csrc", f)).read()
                  for f in os.listdir(os.path.join(ROOT, "aicp_mapping_amd", "csrc"))
                  if f.endswith((".cpp", ".hip", ".hpp")))
    assert "getenv" not in src


def test_parse_default_chain_fixture(L):
    rc, c = L.parse_pm_yaml(os.path.join(GOLDEN, "icp_autotuned_default.yaml"))
    assert rc == 0
    d = L.default_config()
    for k, _ in L.IcpConfig._fields_:
        assert getattr(c, k) == getattr(d, k), k


def _chain(tmp_path, name, minimizer="PointToPlaneErrorMinimizer", outlier="TrimmedDistOutlierFilter",
           ratio="0.55", eps="3.16", knn_normals="20", checkers=True):
    txt = f"""readingDataPointsFilters:
  - SurfaceNormalDataPointsFilter:
        knn: {knn_normals}
        keepDensities: 1
referenceDataPointsFilters:
  - SurfaceNormalDataPointsFilter:
        knn: {knn_normals}
        keepDensities: 1
matcher:
  KDTreeMatcher:
    knn: 1
    epsilon: {eps}
outlierFilters:
  - {outlier}:
      ratio: {ratio}
errorMinimizer:
  {minimizer}:
transformationCheckers:
"""
    if checkers:
        txt += """  - CounterTransformationChecker:
      maxIterationCount: 30
  - DifferentialTransformationChecker:
      minDiffRotErr: 0.002
      minDiffTransErr: 0.02
      smoothLength: 3
"""
    txt += "inspector:\n  NullInspector\nlogger:\n  NullLogger\n"
    p = tmp_path / name
    p.write_text(txt)
    return str(p)


def test_parse_chain_values(L, tmp_path):
    rc, c = L.parse_pm_yaml(_chain(tmp_path, "a.yaml", ratio="0.55", eps="1.5", knn_normals="10"))
    assert rc == 0
    assert c.trimmed_ratio == np.float32(0.55) and c.nn_epsilon == np.float32(1.5) and c.knn_normals == 10
    assert (c.max_iter, c.smooth_length) == (30, 3)
    assert c.min_diff_rot == np.float32(0.002) and c.min_diff_trans == np.float32(0.02)


@pytest.mark.parametrize("kw", [dict(minimizer="PointToPointErrorMinimizer"),
                                dict(outlier="MaxDistOutlierFilter")])
def test_parse_unsupported_chain(L, tmp_path, kw):
    rc, _ = L.parse_pm_yaml(_chain(tmp_path, "u.yaml", **kw))
    assert rc == L.AICP_ERR_UNSUPPORTED


def test_parse_missing_file(L, tmp_path):
    rc, _ = L.parse_pm_yaml(str(tmp_path / "nope.yaml"))
    assert rc == L.AICP_ERR_INVALID


def _fmt6(r):
    # std::ostream << float: %g with 6 significant digits (fileIO.cpp:194-208)
    return "%g" % np.float32(r)


@pytest.mark.parametrize("r", [0.25, 0.7, 0.5, 0.3588, 0.123456789, 0.6999999])
def test_replace_ratio_byte_exact(L, tmp_path, r):
    src = os.path.join(GOLDEN, "icp_autotuned_default.yaml")
    out = tmp_path / "out.yaml"
    rc = L.replace_ratio_config_file(src, str(out), float(np.float32(r)))
    assert rc == 0
    # fileIO.cpp:179-214: `while (!eof) { getline; replace "ratio: " + 4 chars; out << line << "\n"; }`
    # -- every matching line, and one extra newline after the final (empty) getline
    key = b"ratio: "
    lines = []
    for line in open(src, "rb").read().split(b"\n"):
        i = line.find(key)
        if i >= 0:
            line = line[:i] + key + _fmt6(r).encode() + line[i + len(key) + 4:]
        lines.append(line + b"\n")
    assert out.read_bytes() == b"".join(lines)
    rc2, c = L.parse_pm_yaml(str(out))
    assert rc2 == 0 and c.trimmed_ratio == np.float32(float(_fmt6(r)))


def test_autotune_ratio_matches_app_rule(L, oracle):
    # app.cpp:197-205: clamp(overlap / 100, 0.25, 0.70), then the text round trip of a2
    for ov in list(np.linspace(-5, 105, 221)) + [25.0, 70.0, 33.333333, 66.66667, 0.0, 100.0]:
        r = np.float32(min(max(np.float32(ov) / np.float32(100.0), np.float32(0.25)), np.float32(0.70)))
        expect = np.float32(float(_fmt6(r)))
        assert L.autotune_ratio(float(ov)) == expect, ov
        assert oracle.autotune_ratio(float(ov)) == expect, ov


def test_create_reports_hip_error_without_gpu(L):
    if os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK | os.W_OK):
        pytest.skip("a GPU node is present")
    h = C.c_void_p()
    rc = L.lib.aicp_hip_create(0, C.byref(h))
    assert rc == L.AICP_ERR_HIP
    assert not h.value


# ---------------------------------------------------------------------------------------------
# multi-rank plumbing (gloo, world_size 2)
# ---------------------------------------------------------------------------------------------
def test_shard_pairs_partition():
    from aicp_mapping_amd import sharding as sh

    for world in (1, 2, 3, 8):
        got = sorted(i for g in range(world) for i in sh.shard_pairs(37, world, g))
        assert got == list(range(37))
    w = np.arange(1, 11, dtype=float)
    shards = [sh.shard_pairs(10, 2, g, weights=w) for g in range(2)]
    assert sorted(shards[0] + shards[1]) == list(range(10))
    loads = [w[s].sum() for s in shards]
    assert abs(loads[0] - loads[1]) <= w.max()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q, n_pairs):
    import torch.distributed as dist

    from aicp_mapping_amd import sharding as sh

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        idx = sh.shard_pairs(n_pairs, world, rank)
        T = np.stack([np.eye(4, dtype=np.float32).T.reshape(-1) + i for i in idx])
        rec = sh.pack_records(T, [10 + i for i in idx], [0.5 + 0.01 * i for i in idx])
        by_index = sh.gather_records(rec, dist, pair_index=idx)
        rank_major = sh.gather_records(rec, dist)
        m = sh.max_over_ranks(float(rank + 1), dist)
        s = sh.sum_over_ranks(float(rank + 1), dist)
        q.put((rank, by_index, rank_major, m, s))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("n_pairs", [6, 5])
def test_gloo_world2_gather_records(n_pairs):
    """Result records of independent pairs gathered over 2 ranks, also when the i mod G split
    leaves the ranks with different pair counts (5 pairs: 3 + 2, padded for the collective)."""
    import torch.multiprocessing as mp

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, n_pairs)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for rank, by_index, rank_major, m, s in res:
        assert by_index.shape == (n_pairs, 18) and rank_major.shape == (n_pairs, 18)
        # with the shard's pair indices: global pair order
        np.testing.assert_array_equal(by_index[:, 16], [10 + i for i in range(n_pairs)])
        np.testing.assert_allclose(by_index[:, 0], [1 + i for i in range(n_pairs)])
        np.testing.assert_allclose(by_index[:, 17], [0.5 + 0.01 * i for i in range(n_pairs)], rtol=1e-6)
        # default: rank-major (rank 0's pairs 0, 2, 4, then rank 1's 1, 3, ...)
        order = list(range(0, n_pairs, 2)) + list(range(1, n_pairs, 2))
        np.testing.assert_array_equal(rank_major[:, 16], [10 + i for i in order])
        assert m == 2.0 and s == 3.0


def test_as_points_pcl_layouts(L):
    """PointXYZ (16 B), PointXYZRGB (32 B) and PointXYZRGBNormal (48 B) rows pass through with
    their stride; other widths are refused."""
    import numpy as np

    for w in (3, 4, 8, 12):
        a = np.zeros((5, w), np.float32)
        assert L.as_points(a) is a
    for w in (2, 5, 16):
        with pytest.raises(ValueError):
            L.as_points(np.zeros((5, w), np.float32))


def test_xyzrgbnormal_register_is_reference_noop():
    """registerClouds over PointXYZRGBNormal rows leaves final_transform unchanged, as the
    reference's commented-out overload does (pointmatcher_registration.cpp:35-44); no device
    work is started (runs without a GPU)."""
    from aicp_mapping_amd import registration as R

    reg = R.create_registrator(R.RegistrationParams(type="HIP"))
    pts = np.zeros((100, 12), np.float32)
    T = np.arange(16, dtype=np.float32).reshape(4, 4)
    out = reg.registerClouds(pts, pts, T)
    assert out is T and np.array_equal(T, np.arange(16, dtype=np.float32).reshape(4, 4))
    assert reg.registerClouds(pts, pts) is None
    assert reg._ctx is None


@pytest.mark.parametrize("seed", [0, 1, 2, 3])
def test_isometry_from_matrix4f_matches_oracle(oracle, seed):
    """registration.isometry_from_matrix4f (fromMatrix4fToIsometry3d, common.cpp:4-23) moves a
    prior origin like the oracle's corrected_origin, across the quaternion's trace and
    largest-diagonal branches (seeds 2, 3: rotations near pi)."""
    from aicp_mapping_amd import registration as R
    from aicp_mapping_amd import synthetic as sy

    rng = np.random.default_rng(seed)
    yaw = [10.0, -35.0, 179.0, -178.5][seed]
    T = sy.make_T(yaw_deg=yaw, pitch_deg=rng.uniform(-5, 5), roll_deg=rng.uniform(-5, 5),
                  t=rng.uniform(-3, 3, 3)).astype(np.float32)
    o = rng.uniform(-20, 20, 3)
    got = (R.isometry_from_matrix4f(T) @ np.r_[o, 1.0])[:3]
    np.testing.assert_allclose(got, oracle.corrected_origin(T, o), rtol=0, atol=1e-12)
