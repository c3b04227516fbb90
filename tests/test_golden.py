"""Golden vectors (tests/golden/*.npz, made by tests/golden/make_golden.py from the oracle).

CPU: the oracle still reproduces them exactly (it is the parity anchor, so it must not drift).
GPU: the device reproduces them -- bit-exact for ids, d2, counts, limits and iteration counts,
1e-6 rad / 1e-5 m for transforms (the north-star bar is 1e-4 rad / 1e-3 m).
"""
import os

import numpy as np
import pytest

from aicp_mapping_amd import synthetic as sy

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def load(name):
    return np.load(os.path.join(G, name + ".npz"))  # allow_pickle=False (default)


def icp_cases():
    d = load("icp")
    out = []
    for n in d["names"]:
        n = str(n)
        if n == "cube":
            ref = sy.make_cube()
            read = sy.transform(np.linalg.inv(d["cube__perturbation"]), ref).astype(np.float32)
        else:
            ref, read = d[n + "__ref"], d[n + "__read"]
        T0 = d[n + "__T0"]
        out.append(dict(name=n, ref=ref, read=read, ratio=float(d[n + "__ratio"]),
                        T0=None if np.array_equal(T0, np.eye(4, dtype=np.float32)) else T0,
                        rc=int(d[n + "__rc"]), T=d[n + "__T"], iterations=int(d[n + "__iterations"]),
                        inlier_ratio=float(d[n + "__inlier_ratio"])))
    return out


# ------------------------------------------------------------------------------ oracle (CPU)
def test_oracle_knn_golden(oracle):
    d = load("knn")
    t = oracle.Tree(d["ref"])
    ids, d2, tp, tn = t.knn(d["queries"], k=1, eps=3.16)
    np.testing.assert_array_equal(ids, d["ids_k1_eps316"])
    np.testing.assert_array_equal(d2, d["d2_k1_eps316"])
    assert [tp, tn] == list(d["touched_k1"])
    ids, d2, tp, tn = t.knn(d["ref"][:500], k=20, eps=0.0)
    np.testing.assert_array_equal(ids, d["ids_k20"])
    np.testing.assert_array_equal(d2, d["d2_k20"])


def test_oracle_normals_golden(oracle):
    d = load("normals")
    nrm, _, deg = oracle.surface_normals(d["pts"], 20)
    np.testing.assert_array_equal(nrm, d["normals"])
    assert deg == int(d["degenerate"])


def test_oracle_quantile_solve_overlap_golden(oracle):
    q = load("quantile")
    for r, lim in zip(q["ratios"], q["limits"]):
        assert oracle.dists_quantile(q["d2"], float(r))[0] == lim
    s = load("solve6")
    for A, b, x, path in zip(s["A"], s["b"], s["x"], s["path"]):
        x2, p2 = oracle.solve6(A, b)
        np.testing.assert_array_equal(x2, x)
        assert p2 == path
    o = load("overlap")
    ov, cnt = oracle.overlap(o["ref"], o["ref_origin"], o["read"], o["read_origin"], float(o["resolution"]))
    np.testing.assert_array_equal(cnt, o["counts"])
    assert np.float32(ov) == o["overlap"]
    assert np.float32(oracle.autotune_ratio(ov)) == o["ratio"]


@pytest.mark.parametrize("case", icp_cases(), ids=lambda c: c["name"])
def test_oracle_icp_golden(oracle, case):
    rc, T, st = oracle.icp(case["ref"], case["read"], oracle.default_config(trimmed_ratio=case["ratio"]),
                           T0=case["T0"])
    assert rc == case["rc"]
    np.testing.assert_array_equal(T.astype(np.float32), case["T"])
    assert st.iterations == case["iterations"]


# ------------------------------------------------------------------------------ device (GPU)
@pytest.fixture(scope="module")
def ctx():
    import aicp_mapping_amd._lib as L

    c = L.Context(0)
    yield c
    c.close()


@pytest.mark.gpu
def test_device_knn_golden(ctx):
    d = load("knn")
    ids, d2, tp = ctx.knn(d["ref"], d["queries"], k=1, eps=3.16)[:3]
    np.testing.assert_array_equal(ids, d["ids_k1_eps316"])
    np.testing.assert_array_equal(d2, d["d2_k1_eps316"])
    assert tp == int(d["touched_k1"][0])
    ids, d2 = ctx.knn(d["ref"], d["ref"][:500], k=20, eps=0.0)[:2]
    np.testing.assert_array_equal(ids, d["ids_k20"])
    np.testing.assert_array_equal(d2, d["d2_k20"])


@pytest.mark.gpu
def test_device_normals_quantile_solve_golden(ctx):
    d = load("normals")
    nrm, deg = ctx.normals(d["pts"], 20)
    dots = np.abs(np.sum(nrm.astype(np.float64) * d["normals"], 1))  # eigenvector sign is free
    assert np.all(dots > 1 - 1e-6), dots.min()
    assert deg == int(d["degenerate"])
    q = load("quantile")
    for r, lim in zip(q["ratios"], q["limits"]):
        assert ctx.dists_quantile(q["d2"], float(r)) == lim
    s = load("solve6")
    for A, b, x, path in zip(s["A"], s["b"], s["x"], s["path"]):
        x2, p2 = ctx.solve6(A, b)
        np.testing.assert_allclose(x2, x, rtol=1e-9, atol=1e-12)
        assert p2 == path


@pytest.mark.gpu
def test_device_overlap_golden(ctx):
    import aicp_mapping_amd._lib as L

    o = load("overlap")
    _, st, _ = ctx.align_batch([dict(ref=o["ref"], read=o["read"], ref_origin=o["ref_origin"],
                                     read_origin=o["read_origin"])], flags=L.AICP_RUN_OVERLAP,
                               resolution=float(o["resolution"]))
    assert st[0]["overlap_keys"] == [int(c) for c in o["counts"]]
    assert np.float32(st[0]["overlap_percent"]) == o["overlap"]


@pytest.mark.gpu
@pytest.mark.parametrize("case", icp_cases(), ids=lambda c: c["name"])
def test_device_icp_golden(ctx, case):
    import aicp_mapping_amd._lib as L

    cfg = L.default_config(trimmed_ratio=case["ratio"])
    T, st, rc = ctx.align_batch([dict(ref=case["ref"], read=case["read"], init_T=case["T0"])], cfg,
                                flags=L.AICP_RUN_ICP, raise_on_error=False)
    assert rc == case["rc"]
    r, t = sy.rot_err(case["T"], T[0])
    assert r < 1e-6 and t < 1e-5, (r, t)
    assert st[0]["iterations"] == case["iterations"]
