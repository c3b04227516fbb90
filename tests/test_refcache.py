"""The drop-in path's reference cache (runtime.hpp: RefCache; include/aicp_hip.h,
aicp_hip_reference_cache_stats).

App registers reading after reading against one reference (app.cpp:72-73; a new one every
reference_update_frequency readings, app.cpp:383-391) and calls computeOverlap then registerClouds
for each (app.cpp:132-135, 205-210). The one-shot C-ABI calls keep that reference's centroid,
kd-trees, treelets, normals and voxel map resident and reuse them while the same reference array
comes back with the same points. These tests check that the reuse changes no result (transforms,
statistics, key counts bit for bit against a context that rebuilds everything), that it happens
(the hit counters), and that an in-place change of the reference, a new origin or resolution, a
new chain or another call in between makes the next call rebuild.
"""
import numpy as np
import pytest

from aicp_mapping_amd import synthetic as sy

pytestmark = pytest.mark.gpu
RES = float(np.float32(0.2))


@pytest.fixture(scope="module")
def L():
    import aicp_mapping_amd._lib as L

    return L


def _window(seed=21, n=5000, k=5):
    st = sy.make_stream(n_readings=k, n_points=n, seed=seed, half=18.0)
    return st.first, st.first_origin, st.readings, st.origins


def _app_reading(ctx, L, ref, ref_origin, read, read_origin):
    """One reading as App runs it: computeOverlap, the auto-tuned ratio, registerClouds."""
    ov = ctx.overlap(ref, read, ref_origin, read_origin, RES)
    cfg = L.default_config(trimmed_ratio=L.autotune_ratio(ov))
    T, st = ctx.register(ref, read, cfg)
    return ov, T, st


def test_app_pattern_reuses_the_reference_and_matches_cold_runs(L):
    ref, ro, reads, origins = _window()
    warm = L.Context(0)
    got = [_app_reading(warm, L, ref, ro, r, o) for r, o in zip(reads, origins)]
    s = warm.reference_cache_stats()
    assert (s["tree_builds"], s["tree_hits"]) == (1, len(reads) - 1), s
    assert (s["ovl_builds"], s["ovl_hits"]) == (1, len(reads) - 1), s
    for (ov, T, st), r, o in zip(got, reads, origins):
        cold = L.Context(0)  # a new context builds the reference side for this reading alone
        ov1, T1, st1 = _app_reading(cold, L, ref, ro, r, o)
        cold.close()
        assert ov == ov1
        np.testing.assert_array_equal(T, T1)
        assert st == st1
    warm.close()


def test_cached_reference_matches_oracle(L, oracle):
    ref, ro, reads, origins = _window(seed=22, k=3)
    ctx = L.Context(0)
    for r, o in zip(reads, origins):
        ov, T, st = _app_reading(ctx, L, ref, ro, r, o)
        ov_o, cnt = oracle.overlap(ref, ro, r, o, RES)
        assert np.float32(ov) == np.float32(ov_o), (ov, ov_o)
        ratio = oracle.autotune_ratio(ov_o)
        assert np.float32(L.autotune_ratio(ov)) == np.float32(ratio)
        rc1, T1, st1 = oracle.icp(ref, r, oracle.default_config(trimmed_ratio=ratio))
        rr, tt = sy.rot_err(T1, T)
        assert rc1 == 0 and rr < 1e-6 and tt < 1e-5, (rr, tt)
        assert st["iterations"] == st1.iterations
        assert (st["nn_points_touched"], st["nn_nodes_touched"]) == (st1.nn_points_touched, st1.nn_nodes_touched)
    assert ctx.reference_cache_stats()["tree_hits"] == len(reads) - 1
    ctx.close()


def test_in_place_change_of_the_reference_is_seen(L):
    """The reference array is rewritten in place between two calls (same pointer, count and
    stride): the byte compare sees it, and the next call equals a cold context's result."""
    ref, ro, reads, origins = _window(seed=23, k=2)
    ref = ref.copy()
    ctx = L.Context(0)
    ctx.register(ref, reads[0])
    ref[::7] += np.float32(0.05)  # the same buffer, other points
    T, st = ctx.register(ref, reads[1])
    s = ctx.reference_cache_stats()
    assert (s["tree_builds"], s["tree_hits"]) == (2, 0), s
    cold = L.Context(0)
    T1, st1 = cold.register(ref, reads[1])
    cold.close()
    np.testing.assert_array_equal(T, T1)
    assert st == st1
    T2, _ = ctx.register(ref, reads[1])  # now cached: a hit, the same result
    np.testing.assert_array_equal(T, T2)
    assert ctx.reference_cache_stats()["tree_hits"] == 1
    ctx.close()


def test_what_invalidates_the_cache(L):
    """A new origin or resolution rebuilds the voxel map only; another chain's bucket size, a
    call with several references or a kernel-level call rebuilds the trees."""
    ref, ro, reads, origins = _window(seed=24, k=2)
    ctx = L.Context(0)
    ov0 = ctx.overlap(ref, reads[0], ro, origins[0], RES)
    assert ctx.overlap(ref, reads[0], ro, origins[0], RES) == ov0  # hit
    ctx.overlap(ref, reads[0], np.asarray(ro) + 0.5, origins[0], RES)  # new origin
    ctx.overlap(ref, reads[0], np.asarray(ro) + 0.5, origins[0], float(np.float32(0.25)))  # new resolution
    s = ctx.reference_cache_stats()
    assert (s["ovl_builds"], s["ovl_hits"]) == (3, 1), s
    T0, _ = ctx.register(ref, reads[0])
    T1, _ = ctx.register(ref, reads[0], L.default_config(bucket_size=6))  # another tree
    T2, _ = ctx.register(ref, reads[0])  # (rebuilt for bucket 8)
    ctx.align_batch([dict(ref=ref, read=reads[0]), dict(ref=reads[1], read=reads[0])])  # two references
    T3, _ = ctx.register(ref, reads[0])
    ctx.knn(ref, reads[0], 1)  # the kernel-level kNN rewrites the tree buffers
    T4, _ = ctx.register(ref, reads[0])
    s = ctx.reference_cache_stats()
    assert s["tree_hits"] == 0 and s["tree_builds"] >= 5, s
    for T in (T2, T3, T4):
        np.testing.assert_array_equal(T, T0)
    assert ctx.overlap(ref, reads[1], ro, origins[1], RES) == ctx.overlap(ref, reads[1], ro, origins[1], RES)
    ctx.close()


def test_reading_reused_between_overlap_and_register(L):
    """registerClouds after computeOverlap with the same reading array reuses its upload and
    Morton order (ReadCache); a reading rewritten in place between the two calls is uploaded
    again. Every result equals a cold context's."""
    ref, ro, reads, origins = _window(seed=25, k=2)
    r = reads[0].copy()
    ctx = L.Context(0)
    ov, T, st = _app_reading(ctx, L, ref, ro, r, origins[0])
    cold = L.Context(0)
    ov1, T1, st1 = _app_reading(cold, L, ref, ro, r, origins[0])
    np.testing.assert_array_equal(T, T1)
    assert ov == ov1 and st == st1
    ctx.overlap(ref, r, ro, origins[0], RES)
    r[::5] += np.float32(0.02)  # rewritten in place after the overlap call
    T2, st2 = ctx.register(ref, r, L.default_config(trimmed_ratio=L.autotune_ratio(ov)))
    T3, st3 = cold.register(ref, r, L.default_config(trimmed_ratio=L.autotune_ratio(ov)))
    np.testing.assert_array_equal(T2, T3)
    assert st2 == st3
    cold.close()
    ctx.close()
