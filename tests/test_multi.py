"""aicp_hip_multi (multi.cpp): independent pairs sharded over several contexts, one host thread
each, results gathered at the pairs' own indices (SURVEY §8(e), C5's split for a C++ host).

The box has one GPU, so the shards are contexts listed on device 0 more than once: the sharding,
the threads and the gather are the same code as on 8 devices. A pair's result does not depend on
its batch, so every transform, statistic and status must equal one context's align_batch over
all pairs, bit for bit.
"""
import numpy as np
import pytest

from aicp_mapping_amd import synthetic as sy

RES = float(np.float32(0.2))


@pytest.fixture(scope="module")
def L():
    import aicp_mapping_amd._lib as L

    return L


def _pairs(n, seed0):
    # unequal sizes, so the longest-processing-time shards differ in pair count
    prs = [sy.make_pair(6000 + 3000 * (i % 3), 7000 + 2000 * (i % 4), seed=seed0 + i) for i in range(n)]
    return [dict(ref=p.ref, read=p.read, ref_origin=p.ref_origin, read_origin=p.read_origin) for p in prs]


@pytest.mark.gpu
@pytest.mark.parametrize("shards", [1, 3])
def test_multi_align_batch_equals_one_context(L, shards):
    pairs = _pairs(7, 400)
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
    c = L.Context(0)
    T1, s1, rc1 = c.align_batch(pairs, flags=flags, resolution=RES)
    c.close()
    assert rc1 == 0
    m = L.MultiContext(devices=[0] * shards)
    assert m.size() == shards
    Tm, sm, dev, rcm = m.align_batch(pairs, flags=flags, resolution=RES)
    m.close()
    assert rcm == 0
    np.testing.assert_array_equal(Tm, T1)
    assert sm == s1
    assert (dev == 0).all()


@pytest.mark.gpu
def test_multi_default_devices_and_empty_batch(L):
    m = L.MultiContext(n_devices=1)
    assert m.size() == 1
    T, s, dev, rc = m.align_batch([], flags=L.AICP_RUN_ICP)
    assert rc == 0 and T.shape == (0, 4, 4) and s == []
    m.close()


@pytest.mark.gpu
def test_multi_rejects_bad_device(L):
    with pytest.raises(L.AicpError):
        L.MultiContext(devices=[0, 1 << 20])
