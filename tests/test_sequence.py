"""App's frame-to-reference stream on the device (aicp_hip_sequence_run) against the oracle's
replay of App::processCloud (oracle/pyoracle.py: sequence).

The reference builds every reference after the first from a corrected reading (app.cpp:366-391):
reading 5j+4 (when all are accepted) is transformed by its own correction and becomes the
reference of the next window, with the corrected pose's translation as its sensor origin. The
device does that without a host round trip; these tests check that every reading sees the same
reference as in the oracle's sequential replay: overlap key counts bit-exact, transforms within
1e-6 rad / 1e-5 m, iteration counts equal, and the same drop / reference-update decisions.
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


@pytest.fixture(scope="module")
def ctx(L):
    c = L.Context(0)
    yield c
    c.close()


def _compare(out, ref, T, tol_rot=1e-6, tol_t=1e-5):
    assert len(out) == len(ref)
    for i, (o, r) in enumerate(zip(out, ref)):
        assert o["status"] == r["status"], i
        if o["status"]:
            continue
        assert o["reference"] == r["reference"], (i, o["reference"], r["reference"])
        assert o["accepted"] == r["accepted"], i
        assert o["is_reference"] == r["is_reference"], i
        if "counts" in r:
            assert o["icp"]["overlap_keys"] == [int(c) for c in r["counts"]], i
            assert o["icp"]["trimmed_ratio"] == np.float32(r["ratio"]), i
        assert o["icp"]["iterations"] == r["stats"].iterations, i
        rr, tt = sy.rot_err(r["T"], T[i])
        assert rr < tol_rot and tt < tol_t, (i, rr, tt)
        if r["accepted"]:
            np.testing.assert_allclose(o["corrected_origin"], r["corrected_origin"], rtol=0, atol=1e-9)


@pytest.mark.parametrize("freq,n_read", [(5, 12), (3, 7), (1, 4)])
def test_sequence_matches_oracle_replay(ctx, oracle, L, freq, n_read):
    st = sy.make_stream(n_readings=n_read, n_points=5000, seed=7, half=18.0)
    prm = L.default_sequence_params(reference_update_frequency=freq)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    assert rc == 0 and done == n_read
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins, reference_update_frequency=freq,
                          resolution=RES)
    _compare(out, ref, T)
    # every reading of window j > 0 was registered against reading freq*j - 1 (all accepted)
    assert [o["reference"] for o in out] == [-1 if i < freq else (i // freq) * freq - 1 for i in range(n_read)]
    tm = ctx.last_sequence_timing()
    assert tm["windows"] == (n_read + freq - 1) // freq and tm["replans"] == 0
    for i, Tg in enumerate(st.T_gt):
        rg, tg = sy.rot_err(Tg, T[i])
        assert rg < 3e-3 and tg < 3e-2, (i, rg, tg)


def test_sequence_drops_and_replans(ctx, oracle, L):
    """Readings 2 and 6 carry a 0.6 m odometry jump: their corrections exceed
    max_correction_magnitude 0.4, App drops them (app.cpp:366-373) and the window waits for
    more readings, so the reference updates move (reading 5 closes window 0, reading 11 window 1).
    The device's speculative schedule detects both and re-plans from there."""
    st = sy.make_stream(n_readings=12, n_points=5000, seed=8, half=18.0, jumps={2: (0.6, 0, 0), 6: (0, -0.6, 0)})
    prm = L.default_sequence_params(max_correction_magnitude=0.4)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins, max_correction_magnitude=0.4,
                          resolution=RES)
    assert rc == 0 and done == 12
    assert [r["accepted"] for r in ref] == [1, 1, 0, 1, 1, 1, 0, 1, 1, 1, 1, 1]
    _compare(out, ref, T)
    assert [i for i, o in enumerate(out) if o["is_reference"]] == [5, 11]
    assert ctx.last_sequence_timing()["replans"] == 2


def test_sequence_error_ends_stream(ctx, oracle, L):
    """A registration error ends App's worker (uncaught PM::ConvergenceError, app.cpp:210): the
    stream stops at that reading and nothing after it is reported."""
    st = sy.make_stream(n_readings=9, n_points=4000, seed=9, half=15.0)
    st.readings[6] = (st.readings[6] + np.float32(200.0)).astype(np.float32)
    st.origins[6] = st.origins[6] + 200.0
    cfg = L.default_config(nn_max_dist=5.0)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, cfg=cfg,
                                        raise_on_error=False)
    ocfg = oracle.default_config(nn_max_dist=5.0)
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins, cfg=ocfg, resolution=RES)
    assert rc == L.AICP_ERR_CONVERGENCE and done == 7 and len(ref) == 7 and ref[-1]["status"] == 1
    _compare(out, ref, T)
    with pytest.raises(L.ConvergenceError):
        ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, cfg=cfg)


def test_sequence_fixed_ratio_and_layouts(ctx, oracle, L):
    """Without the overlap (AICP_RUN_OVERLAP off) every reading runs at cfg's ratio; PointXYZ rows
    (16 B) give the packed-xyz result bit for bit."""
    st = sy.make_stream(n_readings=6, n_points=4000, seed=10, half=15.0)
    prm = L.default_sequence_params(flags=0)
    cfg = L.default_config(trimmed_ratio=0.6)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, cfg=cfg, params=prm)
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins,
                          cfg=oracle.default_config(trimmed_ratio=0.6), overlap=False)
    _compare(out, ref, T)
    pad = lambda a: np.c_[a, np.ones(len(a), np.float32)].astype(np.float32)
    T4, out4, _, _ = ctx.sequence_run(pad(st.first), st.first_origin, [pad(r) for r in st.readings], st.origins,
                                      cfg=cfg, params=prm)
    np.testing.assert_array_equal(T, T4)


def test_sequence_repeatable_and_matches_batch_window0(ctx, L):
    """Two runs give identical corrections; the readings of the first window equal a batch run of
    the same pairs (the first reference is the first cloud itself)."""
    st = sy.make_stream(n_readings=8, n_points=6000, seed=11, half=18.0)
    Ta, oa, _, _ = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins)
    Tb, ob, _, _ = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins)
    np.testing.assert_array_equal(Ta, Tb)
    pairs = [dict(ref=st.first, read=st.readings[i], ref_origin=st.first_origin, read_origin=st.origins[i])
             for i in range(5)]
    Tc, sc, rc = ctx.align_batch(pairs, flags=L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP, resolution=RES)
    np.testing.assert_array_equal(Tc, Ta[:5])
    assert [s["overlap_keys"] for s in sc] == [o["icp"]["overlap_keys"] for o in oa[:5]]


def test_sequence_c2_full_size(ctx, oracle, L):
    """C2 at full size (64 readings of 120k points, a reference every 5): 13 windows, no
    re-plan, all accepted, and readings 0-10 equal the oracle's replay of App's chain
    (app.cpp:375-391, 414): window 0 against the first cloud, window 1 against corrected reading 4
    and reading 10 against corrected reading 9 -- two references built on the device -- with key
    counts, ratios, iterations and decisions exact and T within 1e-6 rad / 1e-5 m. (~7 s of oracle
    time at 1.66 clouds/s.)"""
    st = sy.make_stream(n_readings=64, n_points=120000, seed=1)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins)
    assert rc == 0 and done == 64
    tm = ctx.last_sequence_timing()
    assert tm["windows"] == 13 and tm["replans"] == 0
    assert all(o["accepted"] for o in out)
    assert [i for i, o in enumerate(out) if o["is_reference"]] == list(range(4, 64, 5))
    # the reference chain's own accuracy on this scene (the oracle gives 0.025 rad / 0.13 m on
    # reading 0 too: eps-3.16 matching stalls there, and later windows inherit the reference)
    for i, Tg in enumerate(st.T_gt):
        rg, tg = sy.rot_err(Tg, T[i])
        assert rg < 0.05 and tg < 0.25, (i, rg, tg)
    # oracle: App's chain over readings 0-10 (two device-built references: corrected 4 and 9)
    ref = oracle.sequence(st.first, st.first_origin, st.readings[:11], st.origins[:11], resolution=RES)
    assert [r["reference"] for r in ref] == [-1] * 5 + [4] * 5 + [9]
    _compare(out[:11], ref, T[:11])



def test_sequence_polled_loop_identical(ctx, L):
    """The polled loop (the host stops enqueueing a window's iterations once the update kernel
    reports no active reading) gives the corrections and statistics of the unpolled schedule,
    which runs maxIterationCount launches per window (option no_early_exit = 1), bit for bit,
    across dropped readings and re-plans."""
    st = sy.make_stream(n_readings=12, n_points=5000, seed=8, half=18.0, jumps={2: (0.6, 0, 0), 6: (0, -0.6, 0)})
    prm = L.default_sequence_params(max_correction_magnitude=0.4)  # readings 2 and 6 drop
    with ctx.options(no_early_exit=1):
        T0, out0, done0, rc0 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    T1, out1, done1, rc1 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    assert (rc0, done0) == (rc1, done1) == (0, 12)
    assert sum(1 - o["accepted"] for o in out1) == 2
    assert ctx.last_sequence_timing()["replans"] == 2
    assert np.array_equal(T0, T1)
    for a, b in zip(out0, out1):
        assert a["accepted"] == b["accepted"] and a["reference"] == b["reference"]
        assert a["icp"]["iterations"] == b["icp"]["iterations"]
        assert a["icp"]["nn_points_touched"] == b["icp"]["nn_points_touched"]

def test_sequence_far_return_sparse_overlap(ctx, oracle, L):
    """One lidar return ~5 km away (octomap's insertPointCloud takes any key in range,
    octrees_overlap.cpp:184): in reading 1 (a plain reading) and in reading 4 (window 0's last,
    the source of window 1's reference). Its key box is ~10^10 voxels, so those windows' overlaps
    take the sorted-key path (sequence.cpp, kSeqMapBudget) instead of failing: key counts exact,
    the same decisions and references, transforms within 1e-6 rad / 1e-5 m."""
    st = sy.make_stream(n_readings=10, n_points=5000, seed=12, half=18.0)
    for i in (1, 4):
        far = (np.asarray(st.origins[i], np.float64) + (3000.0, 4000.0, 25.0)).astype(np.float32)
        st.readings[i] = np.r_[st.readings[i], far[None]].astype(np.float32)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins)
    assert rc == 0 and done == 10
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins, resolution=RES)
    _compare(out, ref, T)
    assert [i for i, o in enumerate(out) if o["is_reference"]] == [4, 9]
    # the far ray's keys are in the counts: reading 1's set is ~25k keys larger than its neighbours'
    assert out[1]["icp"]["overlap_keys"][1] > out[0]["icp"]["overlap_keys"][1] + 20000


def test_sequence_sparse_overlap_identical(ctx, L):
    """Every window on the sorted-key path (option overlap_path = 1) gives the dense maps' key counts
    and corrections bit for bit, across dropped readings and re-plans."""
    st = sy.make_stream(n_readings=12, n_points=5000, seed=8, half=18.0, jumps={2: (0.6, 0, 0), 6: (0, -0.6, 0)})
    prm = L.default_sequence_params(max_correction_magnitude=0.4)
    T0, out0, done0, rc0 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    with ctx.options(overlap_path=1):
        T1, out1, done1, rc1 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    assert (rc0, done0) == (rc1, done1) == (0, 12)
    assert np.array_equal(T0, T1)
    for a, b in zip(out0, out1):
        assert a["icp"]["overlap_keys"] == b["icp"]["overlap_keys"]
        assert a["accepted"] == b["accepted"] and a["reference"] == b["reference"]


@pytest.mark.parametrize("jumps", [None, {2: (0.6, 0, 0), 6: (0, -0.6, 0)}])
def test_sequence_debug_mode_matches_oracle(ctx, oracle, L, jumps):
    """App's "debug" working mode (aicp.launch:36; app.cpp:87-96, 414): every reading is first
    moved by initialT_ (the product of the accepted corrections so far) and its prior pose with
    it; a dropped reading leaves initialT_ as it was. The device registers the readings of a
    window one after the other against the window's reference; the corrections, decisions,
    references, corrected poses and key counts equal the oracle's replay of the same mode."""
    st = sy.make_stream(n_readings=12, n_points=5000, seed=8, half=18.0, jumps=jumps)
    prm = L.default_sequence_params(max_correction_magnitude=0.4, flags=L.AICP_RUN_OVERLAP | L.AICP_SEQ_DEBUG)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    assert rc == 0 and done == 12
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins, max_correction_magnitude=0.4,
                          resolution=RES, working_mode="debug")
    _compare(out, ref, T)
    assert ctx.last_sequence_timing()["replans"] == (2 if jumps else 0)
    # after the first correction initialT_ carries the drift: the later corrections are small
    if not jumps:
        for i in range(2, 12):
            rr, tt = sy.rot_err(np.eye(4), T[i])
            assert rr < 5e-3 and tt < 5e-2, (i, rr, tt)


def test_sequence_debug_mode_sparse_overlap(ctx, oracle, L):
    """Debug mode with every overlap on the sorted-key path (one key side per reading, bounds for
    any rigid motion): the same results as the dense maps, and the oracle's."""
    st = sy.make_stream(n_readings=7, n_points=4000, seed=9, half=15.0)
    prm = L.default_sequence_params(flags=L.AICP_RUN_OVERLAP | L.AICP_SEQ_DEBUG)
    T0, out0, _, rc0 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    with ctx.options(overlap_path=1):
        T1, out1, _, rc1 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    assert rc0 == rc1 == 0
    assert np.array_equal(T0, T1)
    assert [o["icp"]["overlap_keys"] for o in out0] == [o["icp"]["overlap_keys"] for o in out1]
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins, resolution=RES, working_mode="debug")
    _compare(out1, ref, T1)


@pytest.mark.parametrize("mode,jumps", [("debug", None), ("debug", {3: (0, -0.8, 0)}), ("robot", None)])
def test_sequence_raw_clouds_in_app_order(ctx, oracle, L, mode, jumps):
    """App's order from RAW clouds (aicp_hip_sequence_run_raw): the first cloud is pre-filtered as
    given (app.cpp:293-297); in debug mode each raw reading is moved by initialT_ and then
    pre-filtered (setAndFilterReading, app.cpp:77-100), in robot mode pre-filtered as given. The
    oracle replays the same order (pcl::transformPointCloud, then its pre-filter restatement):
    decisions, references, key counts, iterations and corrections agree, and the reference's
    trees stay resident across the per-reading pre-filters."""
    st = sy.make_stream(n_readings=10, n_points=20000, seed=8, half=12.0, jumps=jumps)
    flags = L.AICP_RUN_OVERLAP | (L.AICP_SEQ_DEBUG if mode == "debug" else 0)
    prm = L.default_sequence_params(max_correction_magnitude=0.4, flags=flags)
    s0 = ctx.reference_cache_stats()
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm,
                                        prefilter=True)
    s1 = ctx.reference_cache_stats()
    assert rc == 0 and done == 10
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins, max_correction_magnitude=0.4,
                          resolution=RES, working_mode=mode, prefilter_with=True)
    _compare(out, ref, T)
    if jumps:
        assert not out[3]["accepted"] and ref[3]["accepted"] == 0
    if mode == "debug":  # one tree build per reference, every other reading reuses it
        n_refs = len({o["reference"] for o in out})
        assert s1["tree_builds"] - s0["tree_builds"] == n_refs
        assert s1["tree_hits"] - s0["tree_hits"] == 10 - n_refs


@pytest.mark.parametrize("mode", ["debug", "robot"])
def test_sequence_raw_empty_after_prefilter_ends_stream(ctx, oracle, L, mode):
    """A reading the pre-filter empties (30 scattered points: no region of 50) fails its
    registration, which ends the stream there (app.cpp:210); the readings before it are App's."""
    st = sy.make_stream(n_readings=5, n_points=20000, seed=3, half=12.0)
    rng = np.random.default_rng(4)
    reads = st.readings[:3] + [rng.uniform(-5, 5, size=(30, 3)).astype(np.float32)] + st.readings[4:]
    flags = L.AICP_RUN_OVERLAP | (L.AICP_SEQ_DEBUG if mode == "debug" else 0)
    prm = L.default_sequence_params(flags=flags)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, reads, st.origins, params=prm, prefilter=True,
                                        raise_on_error=False)
    assert rc == L.AICP_ERR_INVALID and done == 4
    assert out[3]["status"] == L.AICP_ERR_INVALID and not out[3]["accepted"]
    ref = oracle.sequence(st.first, st.first_origin, reads, st.origins, resolution=RES, working_mode=mode,
                          prefilter_with=True, stop=3)
    _compare(out[:3], ref, T[:3])


def test_sequence_raw_robot_equals_prefilter_then_stream(ctx, L):
    """Robot mode from raw clouds is the device pre-filter of every cloud followed by the stream:
    the same corrections bit for bit as pre-filtering with aicp_hip_prefilter first; invalid
    pre-filter parameters are refused before anything runs."""
    st = sy.make_stream(n_readings=6, n_points=20000, seed=5, half=12.0)
    prm = L.default_sequence_params(flags=L.AICP_RUN_OVERLAP)
    T0, out0, d0, rc0 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm,
                                         prefilter=True)
    kept = [ctx.prefilter(r) for r in st.readings]
    T1, out1, d1, rc1 = ctx.sequence_run(ctx.prefilter(st.first), st.first_origin, kept, st.origins, params=prm)
    assert (rc0, d0) == (rc1, d1) == (0, 6)
    assert np.array_equal(T0, T1)
    assert [o["icp"]["overlap_keys"] for o in out0] == [o["icp"]["overlap_keys"] for o in out1]
    with pytest.raises(L.AicpError):
        ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm,
                         prefilter=L.default_prefilter(normal_k=25))


@pytest.mark.parametrize("jumps", [None, {3: (0, -0.8, 0)}, {4: (0, -0.8, 0)}])
def test_sequence_early_reference_identical(ctx, L, jumps):
    """early_reference (the next window's reference built once its source reading has stopped,
    beside the window's other readings) changes only the schedule: corrections, decisions, key
    counts and iterations equal the whole-window order's bit for bit, drops and re-plans included
    (a dropped source: reading 4 of the first window)."""
    st = sy.make_stream(n_readings=12, n_points=8000, seed=11, half=18.0, jumps=jumps)
    prm = L.default_sequence_params(max_correction_magnitude=0.4)
    T0, out0, d0, rc0 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    with ctx.options(early_reference=0):
        T1, out1, d1, rc1 = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm)
    assert (rc0, d0) == (rc1, d1) == (0, 12)
    assert np.array_equal(T0, T1)
    assert out0 == out1
    if jumps:
        assert not all(o["accepted"] for o in out0)


def test_sequence_raw_debug_c2_full_size(ctx, oracle, L):
    """App's debug order at the C2 size: six raw 120k-point readings moved by initialT_ and
    pre-filtered on the device (~100k points kept each), the fifth corrected into the reference of
    the sixth; the oracle's App-order replay gives the same decisions, key counts, iterations and
    corrections."""
    st = sy.make_stream(n_readings=6, n_points=120000, seed=1, half=30.0)
    prm = L.default_sequence_params(flags=L.AICP_RUN_OVERLAP | L.AICP_SEQ_DEBUG)
    T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, params=prm,
                                        prefilter=True)
    assert rc == 0 and done == 6
    ref = oracle.sequence(st.first, st.first_origin, st.readings, st.origins, resolution=RES, working_mode="debug",
                          prefilter_with=True)
    _compare(out, ref, T)
    assert [o["reference"] for o in out] == [-1] * 5 + [4]
