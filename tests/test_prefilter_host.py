"""Host logic around the device pre-filter and prior map (no GPU): the overload dispatch of
filtering.regionGrowingUniformPlaneSegmentationFilter and App's localization-mode schedule
(app.cpp:469-493) in prior_map.localization_update."""
import numpy as np
import pytest


class FakeCtx:
    def __init__(self):
        self.calls = []

    def prefilter(self, pts, params=None, details=False):
        self.calls.append(("prefilter", details))
        pts = np.asarray(pts, np.float32)[:, :3]
        if not details:
            return pts[::2].copy()
        V = len(pts)
        sampled = np.zeros((V, 8), np.float32)
        sampled[:, :3] = pts
        sampled[:, 3] = 0.01
        sampled[:, 6] = 1.0
        labels = np.where(np.arange(V) % 3 == 0, -1, np.arange(V) % 2).astype(np.int32)
        return dict(out=pts.copy(), sampled=sampled, labels=labels, n_clusters=2)


def test_filter_overloads():
    import aicp_mapping_amd._lib  # noqa: F401  (the library loads without a GPU)
    from aicp_mapping_amd import filtering

    c = FakeCtx()
    P = np.random.default_rng(0).uniform(-1, 1, (30, 3)).astype(np.float32)
    kept = filtering.regionGrowingUniformPlaneSegmentationFilter(P, ctx=c)
    assert np.array_equal(kept, P[::2])
    prev = np.ones((4, 3), np.float32)
    acc = filtering.regionGrowingUniformPlaneSegmentationFilter(P, prev, ctx=c)
    assert np.array_equal(acc[:4], prev) and np.array_equal(acc[4:], P[::2])
    clusters = [np.zeros(3)]
    T = np.eye(4)
    T[:3, 3] = (1.0, 2.0, 3.0)
    out = filtering.regionGrowingUniformPlaneSegmentationFilter(P, T, clusters, ctx=c)
    assert out.shape == (30, 12) and np.array_equal(out[:, :3], P) and np.all(out[:, 3] == 1.0)
    assert len(clusters) == 2
    lab = np.where(np.arange(30) % 3 == 0, -1, np.arange(30) % 2)
    for k in range(2):
        assert np.array_equal(clusters[k], np.nonzero(lab == k)[0])
        assert len(set(out[clusters[k], 8].view(np.uint32).tolist())) == 1  # one colour per cluster
    with pytest.raises(TypeError):
        filtering.regionGrowingUniformPlaneSegmentationFilter(P, T, clusters, 1, ctx=c)


def test_localization_schedule():
    from aicp_mapping_amd.prior_map import localization_update

    class FakeMap:
        def __init__(self):
            self.log = []

        def merge(self, pts, T):
            self.log.append("merge")

        def prefilter(self, params=None):
            self.log.append("prefilter")

    m = FakeMap()
    for n in range(2, 62):
        localization_update(m, None, None, n, reference_update_frequency=5)
    # app.cpp:469-483: (n - 1) % 5 == 0 merges; app.cpp:487-493: (n - 1) % 30 == 0 re-filters
    assert m.log.count("merge") == len([n for n in range(2, 62) if (n - 1) % 5 == 0])
    assert m.log.count("prefilter") == 2
    m2 = FakeMap()
    localization_update(m2, None, None, 31, merge_aligned_clouds_to_map=False)
    assert m2.log == []
