"""Offline input formats: aicp_input_poses.csv, cloud_<c>_<s>_<ns>.pcd
(ascii / binary / binary_compressed) and KITTI .bin, as App::processFromFile reads them
(app.cpp:250-279, poseFileReader.hpp:46-78). CPU tests, plus one GPU test that replays a
recorded directory through the registration mirror and checks it against the oracle.

No PCD or pose file ships in the reference, so the format tests are pinned by hand-made
known-answer streams (LZF control codes, Eigen's quaternion formula) and round trips; the
recorded-directory replay is "parity unpinned" beyond the oracle.
"""
import math
import os
import struct

import numpy as np
import pytest

from aicp_mapping_amd import cloud_io as io
from aicp_mapping_amd import synthetic as sy


def test_lzf_known_answers():
    # literal "abc" then a back-reference of 9 bytes at distance 3 (extended-length form)
    assert io.lzf_decompress(bytes([2, 0x61, 0x62, 0x63, 0xE0, 0x00, 0x02]), 12) == b"abcabcabcabc"
    # literal "a" then a 3-byte overlapping back-reference at distance 1
    assert io.lzf_decompress(bytes([0, 0x61, 0x20, 0x00]), 4) == b"aaaa"
    # empty stream
    assert io.lzf_decompress(b"", 0) == b""
    with pytest.raises(io.CloudFormatError):
        io.lzf_decompress(bytes([0x20, 0x05]), 3)  # back-reference before the start
    with pytest.raises(io.CloudFormatError):
        io.lzf_decompress(bytes([2, 0x61]), 3)  # truncated literal run


def test_lzf_literal_round_trip():
    data = np.random.default_rng(3).integers(0, 256, 1000, dtype=np.uint8).tobytes()
    assert io.lzf_decompress(io.lzf_compress_literal(data), len(data)) == data


@pytest.mark.parametrize("data", ["binary", "ascii", "binary_compressed"])
def test_pcd_round_trip(tmp_path, data):
    P = sy.make_pair(3000, 10, seed=5).ref
    fn = str(tmp_path / f"c_{data}.pcd")
    io.save_pcd_xyz(fn, P, data=data)
    c = io.load_pcd_xyz(fn)
    assert c.width == 3000 and c.height == 1
    assert c.xyz.dtype == np.float32 and np.array_equal(c.xyz, P)  # bit-exact, ascii via repr


def test_pcd_empty_cloud(tmp_path):
    fn = str(tmp_path / "empty.pcd")
    io.save_pcd_xyz(fn, np.zeros((0, 3), np.float32))
    assert io.load_pcd_xyz(fn).xyz.shape == (0, 3)


def test_pcd_extra_fields_organised_and_compressed_soa(tmp_path):
    """x y z among other fields (PointXYZI-style with padding), organised 4x2, stored
    binary_compressed: fields one after another, x/y/z picked by name."""
    w, h = 4, 2
    n = w * h
    rng = np.random.default_rng(9)
    xyz = rng.normal(size=(n, 3)).astype(np.float32)
    inten = rng.integers(0, 255, n).astype(np.uint8)
    ring = rng.integers(0, 16, n).astype(np.uint16)
    raw = inten.tobytes() + xyz[:, 0].tobytes() + xyz[:, 1].tobytes() + ring.tobytes() + xyz[:, 2].tobytes()
    comp = io.lzf_compress_literal(raw)
    head = (f"VERSION 0.7\nFIELDS intensity x y ring z\nSIZE 1 4 4 2 4\nTYPE U F F U F\n"
            f"COUNT 1 1 1 1 1\nWIDTH {w}\nHEIGHT {h}\nVIEWPOINT 1 2 3 1 0 0 0\nPOINTS {n}\n"
            "DATA binary_compressed\n").encode()
    fn = tmp_path / "org.pcd"
    fn.write_bytes(head + struct.pack("<II", len(comp), len(raw)) + comp)
    c = io.load_pcd_xyz(str(fn))
    assert (c.width, c.height) == (w, h) and c.viewpoint[:3] == (1.0, 2.0, 3.0)
    assert np.array_equal(c.xyz, xyz)
    # the same record as AoS binary
    rec = np.zeros(n, dtype=[("intensity", "u1"), ("x", "<f4"), ("y", "<f4"), ("ring", "<u2"), ("z", "<f4")])
    rec["intensity"], rec["x"], rec["y"], rec["ring"], rec["z"] = inten, xyz[:, 0], xyz[:, 1], ring, xyz[:, 2]
    fn2 = tmp_path / "org_bin.pcd"
    fn2.write_bytes(head.replace(b"binary_compressed", b"binary") + rec.tobytes())
    assert np.array_equal(io.load_pcd_xyz(str(fn2)).xyz, xyz)


@pytest.mark.parametrize("bad", [b"VERSION 0.7\nFIELDS x y\nSIZE 4 4\nTYPE F F\nCOUNT 1 1\nWIDTH 1\nHEIGHT 1\nDATA binary\n",
                                 b"FIELDS x y z\nSIZE 4 4 4\nTYPE F F F\nWIDTH 2\nHEIGHT 1\nDATA binary\n" + b"\0" * 12,
                                 b"FIELDS x y z\nSIZE 4 4 4\nTYPE F F F\nWIDTH 1\nHEIGHT 1\nPOINTS 2\nDATA ascii\n1 2 3\n",
                                 b"FIELDS x y z\nSIZE 4 4 4\n"])
def test_pcd_rejects(tmp_path, bad):
    fn = tmp_path / "bad.pcd"
    fn.write_bytes(bad)
    with pytest.raises(io.CloudFormatError):
        io.load_pcd_xyz(str(fn))


def test_quaternion_formula_matches_eigen():
    """Eigen toRotationMatrix for a unit quaternion equals the axis-angle rotation; for a
    non-unit one it is NOT renormalised (reference behaviour)."""
    ang, axis = 0.3, np.array([1.0, 2.0, 2.0]) / 3.0
    w, (x, y, z) = math.cos(ang / 2), math.sin(ang / 2) * axis
    R = io.quat_to_rot(w, x, y, z)
    K = np.array([[0, -axis[2], axis[1]], [axis[2], 0, -axis[0]], [-axis[1], axis[0], 0]])
    R_ref = np.eye(3) + math.sin(ang) * K + (1 - math.cos(ang)) * K @ K
    assert np.allclose(R, R_ref, atol=1e-15)
    assert np.allclose(io.rot_to_quat(R), [w, x, y, z], atol=1e-15)
    R2 = io.quat_to_rot(1.0, 0.1, 0.0, 0.0)  # |q|^2 = 1.01
    assert R2[1, 1] == 1 - 2 * 0.1 * 0.1 and R2[2, 1] == 2 * 0.1 * 1.0


def test_pose_file_reference_semantics(tmp_path):
    fn = tmp_path / "aicp_input_poses.csv"
    fn.write_text("# counter, sec, nsec, x, y, z, qx, qy, qz, qw\n"
                  "0, 1500000000, 250000, 1.5, -2, 0.25, 0, 0, 0.7071068, 0.7071068\n"
                  "1,1500000001,  7, 3e-1 , 0, 0, 0, 0, 0, 1trailing\n")
    ps = io.read_pose_file(str(fn))
    assert [p.counter for p in ps] == [0, 1]
    assert ps[0].sec == 1500000000 and ps[0].nsec == 250000 and ps[0].utime == 1500000000250000
    assert np.allclose(ps[0].pose[:3, 3], [1.5, -2, 0.25])
    assert np.allclose(ps[0].pose[:3, :3] @ [1, 0, 0], [0, 1, 0], atol=1e-7)  # 90 deg yaw
    assert ps[1].pose[0, 3] == 0.3 and np.array_equal(ps[1].pose[:3, :3], np.eye(3))
    assert io.read_pose_file(str(tmp_path / "missing.csv")) == []
    bad = tmp_path / "bad.csv"
    bad.write_text("0, 1, 2, 0, 0, 0, 0, 0, 0, 1\n\n")
    with pytest.raises(io.CloudFormatError):
        io.read_pose_file(str(bad))


def test_pose_line_writer_format():
    T = sy.make_T(yaw_deg=10.0, t=(1.0, 2.0, 3.0))
    line = io.format_pose_line(7, 1500000000123456, T)
    f = [s.strip() for s in line.split(",")]
    assert f[:3] == ["7", "1500000000", "123456"] and f[3:6] == ["1", "2", "3"]
    assert len(f) == 10


def test_kitti_bin(tmp_path):
    rec = np.random.default_rng(1).normal(size=(100, 4)).astype("<f4")
    fn = tmp_path / "000000.bin"
    rec.tofile(fn)
    assert np.array_equal(io.load_kitti_bin(str(fn)), rec[:, :3])
    (tmp_path / "bad.bin").write_bytes(b"\0" * 10)
    with pytest.raises(io.CloudFormatError):
        io.load_kitti_bin(str(tmp_path / "bad.bin"))


def write_recording(d, clouds, poses, t0=1500000000000000):
    recs = []
    for i, (P, T) in enumerate(zip(clouds, poses)):
        rec = io.IsometryWithTime(T, 0, 0, i)
        u = t0 + i * 100000
        rec.sec, rec.nsec = int(math.floor(u * 1e-6)), int(u - math.floor(u * 1e-6) * 1e6)
        io.save_pcd_xyz(io.cloud_file_name(str(d), i, rec.sec, rec.nsec), P)
        recs.append(rec)
    io.write_pose_file(os.path.join(str(d), "aicp_input_poses.csv"), recs)


def test_process_from_file_replay(tmp_path):
    clouds = []
    for k in range(3):
        pr = sy.make_pair(2000, 1500, seed=3 + k)
        clouds += [pr.ref, pr.read]
    poses = [np.eye(4) for _ in clouds]
    write_recording(tmp_path, clouds, poses)
    got = list(io.process_from_file(str(tmp_path)))
    assert len(got) == len(clouds)
    for (p, xyz), P, i in zip(got, clouds, range(len(clouds))):
        assert p.counter == i and np.array_equal(xyz, P)
        assert p.utime == 1500000000000000 + i * 100000
    # a missing cloud stops the replay (app.cpp:269-272)
    os.remove(io.cloud_file_name(str(tmp_path), 2, got[2][0].sec, got[2][0].nsec))
    assert len(list(io.process_from_file(str(tmp_path)))) == 2


@pytest.mark.gpu
def test_recorded_directory_registers_like_oracle(tmp_path, oracle):
    """A recorded pair replayed from disk (binary PCD + pose file) registers through the HIP
    mirror to the oracle's transform."""
    import aicp_mapping_amd._lib as L
    from aicp_mapping_amd import registration as R

    pr = sy.make_pair(6000, 6000, seed=91)
    Pr = np.eye(4); Pr[:3, 3] = pr.ref_origin
    Pd = np.eye(4); Pd[:3, 3] = pr.read_origin
    write_recording(tmp_path, [pr.ref, pr.read], [Pr, Pd])
    (p0, ref), (p1, read) = list(io.process_from_file(str(tmp_path)))
    ctx = L.Context(0)
    try:
        reg = R.RegistrationParams(type="HIP")
        reg.pointmatcher.configFileName = os.path.join(os.path.dirname(__file__), "golden",
                                                       "icp_autotuned_default.yaml")
        pipe = R.AicpPipeline(reg, R.OverlapParams(type="OctreeBased"),
                              registration_config_file=str(tmp_path / "icp.yaml"), ctx=ctx)
        T = pipe.runAicpPipeline(ref, read, p0.pose, p1.pose)
    finally:
        ctx.close()
    ov, _ = oracle.overlap(ref, p0.pose[:3, 3], read, p1.pose[:3, 3], float(np.float32(0.2)))
    assert pipe.octree_overlap_ == np.float32(ov)
    rc, T1, _ = oracle.icp(ref, read, oracle.default_config(trimmed_ratio=oracle.autotune_ratio(ov),
                                                           normals_on_centered=0))
    r, t = sy.rot_err(T1, T)
    assert r < 1e-6 and t < 1e-5


def test_recorded_sequence_pairs_windowing(tmp_path):
    """App's frame-to-reference windowing over a recording: cloud 0 is the first reference;
    the reference moves to the reading that closes every `ref_every` readings."""
    clouds = [sy.make_pair(800, 10, seed=40 + i).ref for i in range(12)]
    poses = []
    for i in range(12):
        T = np.eye(4)
        T[:3, 3] = (0.5 * i, 0.0, 0.7)
        poses.append(T)
    write_recording(tmp_path, clouds, poses)
    pairs = io.recorded_sequence_pairs(str(tmp_path), ref_every=5)
    assert len(pairs) == 11
    ref_idx = [0] * 5 + [5] * 5 + [10]
    for j, (p, r) in enumerate(zip(pairs, ref_idx)):
        assert np.array_equal(p["read"], clouds[j + 1]) and np.array_equal(p["ref"], clouds[r])
        assert np.allclose(p["ref_origin"], (0.5 * r, 0, 0.7)) and p["T_gt"] is None
    # readings of one window share one reference array (the device shares its tree and normals)
    assert len({id(p["ref"]) for p in pairs}) == 3
    assert len(io.recorded_sequence_pairs(str(tmp_path), 5, max_readings=4)) == 4
