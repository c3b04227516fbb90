"""Offline input formats that feed the registration path.

Host-side data plumbing, not compute: it turns the reference's recorded sequences into the
(N, 3) float32 clouds and 4x4 float64 poses that `AicpPipeline` / `aicp_hip_align_batch` take.

Reference formats and the code that reads / writes them (zbqq/aicp_mapping):
  aicp_input_poses.csv   writer  aicp_ros/src/app_ros.cpp:57-62,155-167
                         reader  aicp_core/include/aicp_utils/poseFileReader.hpp:46-78
  cloud_<c>_<s>_<ns>.pcd writer  aicp_ros/src/app_ros.cpp:169-172 (pcl::PCDWriter, binary)
                         reader  aicp_core/src/registration/app.cpp:250-279 (loadPCDFile<PointXYZ>)
  KITTI velodyne .bin    converted by bash/kitti2pcd_no_ground.sh:7-36 (float32 x, y, z, intensity)

PCD support covers what pcl::io::loadPCDFile<PointXYZ> accepts for these files: DATA ascii,
binary and binary_compressed (LZF, fields stored one after another), any field list containing
x, y and z (other fields are skipped, as the PointXYZ field mapping does), organised clouds
(WIDTH x HEIGHT points; the registration path then counts `width` only, cloudIO.cpp:83).
"""
from __future__ import annotations

import os
import struct
from dataclasses import dataclass

import numpy as np

_PCD_NP = {("F", 4): "<f4", ("F", 8): "<f8", ("I", 1): "<i1", ("I", 2): "<i2", ("I", 4): "<i4",
           ("I", 8): "<i8", ("U", 1): "<u1", ("U", 2): "<u2", ("U", 4): "<u4", ("U", 8): "<u8"}


class CloudFormatError(ValueError):
    """A file the reference's loader would reject (loadPCDFile returns -1, app.cpp:269-272)."""


# ----------------------------------------------------------------------------------- poses


@dataclass
class IsometryWithTime:
    """poseFileReader.hpp:20-38: a world-to-body pose with its (sec, nsec) stamp and counter.
    `nsec` holds the microsecond remainder (app_ros.cpp:158-159), so utime = sec*1e6 + nsec
    (app.cpp:266)."""
    pose: np.ndarray  # 4x4 float64
    sec: int
    nsec: int
    counter: int

    @property
    def utime(self) -> int:
        return int(self.sec * 1e6 + self.nsec)


def quat_to_rot(qw, qx, qy, qz) -> np.ndarray:
    """Eigen::Quaterniond::toRotationMatrix: the quaternion is NOT normalised first, so a
    recorded quaternion with rounding error yields the same (slightly non-orthonormal) matrix
    as the reference's `Isometry3d::rotate(Quaterniond(w, x, y, z))` (poseFileReader.hpp:70)."""
    tx, ty, tz = 2 * qx, 2 * qy, 2 * qz
    twx, twy, twz = tx * qw, ty * qw, tz * qw
    txx, txy, txz = tx * qx, ty * qx, tz * qx
    tyy, tyz, tzz = ty * qy, tz * qy, tz * qz
    return np.array([[1 - (tyy + tzz), txy - twz, txz + twy],
                     [txy + twz, 1 - (txx + tzz), tyz - twx],
                     [txz - twy, tyz + twx, 1 - (txx + tyy)]], dtype=np.float64)


def _stod(field: str) -> float:
    """std::stod: leading whitespace skipped, the longest valid prefix parsed, trailing text
    ignored; no valid prefix throws (std::invalid_argument)."""
    s = field.lstrip()
    for end in range(len(s), 0, -1):
        try:
            return float(s[:end])
        except ValueError:
            continue
    raise CloudFormatError(f"stod: no conversion of {field!r}")


def read_pose_file(path: str) -> list[IsometryWithTime]:
    """PoseFileReader::readPoseFile (poseFileReader.hpp:46-78). Lines starting with '#' are
    skipped; every other line is split on ',' and each field parsed with stod; columns are
    counter, sec, nsec, x, y, z, qx, qy, qz, qw. A missing file yields an empty list (the
    reference's `if (in)` guard). An empty line makes the reference throw (`line.at(0)`)."""
    if not os.path.exists(path):
        return []
    out = []
    with open(path, "r") as f:
        lines = f.read().split("\n")
        if lines and lines[-1] == "":
            lines.pop()  # getline does not yield an empty line after the final newline
        for lineno, line in enumerate(lines, 1):
            if line.endswith("\r"):
                line = line[:-1]
            if not line:
                raise CloudFormatError(f"{path}:{lineno}: empty line (std::out_of_range in the reference)")
            if line[0] == "#":
                continue
            row = [_stod(x) for x in line.split(",")]
            if len(row) < 10:
                raise CloudFormatError(f"{path}:{lineno}: {len(row)} fields, 10 expected")
            T = np.eye(4)
            T[:3, 3] = row[3:6]
            T[:3, :3] = quat_to_rot(row[9], row[6], row[7], row[8])
            out.append(IsometryWithTime(T, int(row[1]), int(row[2]), int(row[0])))
    return out


def format_pose_line(counter: int, utime: int, pose: np.ndarray) -> str:
    """One line as AppROS::writeInputCloudToFile writes it (app_ros.cpp:155-166): sec =
    floor(utime*1e-6), nsec = utime - sec*1e6, values via ostream (6 significant digits)."""
    sec = int(np.floor(utime * 1e-6))
    nsec = int(utime - sec * 1e6)
    q = rot_to_quat(np.asarray(pose, dtype=np.float64)[:3, :3])
    t = np.asarray(pose, dtype=np.float64)[:3, 3]
    vals = [f"{v:.6g}" for v in (t[0], t[1], t[2], q[1], q[2], q[3], q[0])]
    return f"{counter}, {sec}, {nsec}, " + ", ".join(vals)


def rot_to_quat(R: np.ndarray) -> np.ndarray:
    """Eigen's Quaterniond(Matrix3d) (Shepperd's method, largest-diagonal branch); returns
    (w, x, y, z)."""
    t = np.trace(R)
    if t > 0:
        s = np.sqrt(t + 1.0)
        w = 0.5 * s
        s = 0.5 / s
        return np.array([w, (R[2, 1] - R[1, 2]) * s, (R[0, 2] - R[2, 0]) * s, (R[1, 0] - R[0, 1]) * s])
    i = int(np.argmax(np.diag(R)))
    j, k = (i + 1) % 3, (i + 2) % 3
    s = np.sqrt(R[i, i] - R[j, j] - R[k, k] + 1.0)
    q = np.zeros(4)
    q[1 + i] = 0.5 * s
    s = 0.5 / s
    q[0] = (R[k, j] - R[j, k]) * s
    q[1 + j] = (R[j, i] + R[i, j]) * s
    q[1 + k] = (R[k, i] + R[i, k]) * s
    return q


def write_pose_file(path: str, poses: list[IsometryWithTime]) -> None:
    """aicp_input_poses.csv with the header line of app_ros.cpp:61."""
    with open(path, "w") as f:
        f.write("# counter, sec, nsec, x, y, z, qx, qy, qz, qw\n")
        for p in poses:
            f.write(format_pose_line(p.counter, p.utime, p.pose) + "\n")


def cloud_file_name(directory: str, counter: int, sec: int, nsec: int) -> str:
    """app.cpp:262-263 / app_ros.cpp:171."""
    return os.path.join(directory, f"cloud_{counter}_{sec}_{nsec}.pcd")


# ------------------------------------------------------------------------------------- LZF


def lzf_decompress(src: bytes, out_len: int) -> bytes:
    """liblzf lzf_decompress (the codec PCL's binary_compressed uses). Control byte c:
    c < 32 -> c+1 literal bytes follow; else a back-reference of length (c >> 5) + 2
    (7 -> 7 + next byte + 2) at distance ((c & 31) << 8 | next byte) + 1. Overlapping copies
    are byte-serial."""
    out = bytearray(out_len)
    ip = op = 0
    n = len(src)
    while ip < n:
        c = src[ip]
        ip += 1
        if c < 32:
            ln = c + 1
            if op + ln > out_len or ip + ln > n:
                raise CloudFormatError("lzf: literal run overflows")
            out[op:op + ln] = src[ip:ip + ln]
            op += ln
            ip += ln
        else:
            ln = c >> 5
            if ln == 7:
                if ip >= n:
                    raise CloudFormatError("lzf: truncated length")
                ln += src[ip]
                ip += 1
            if ip >= n:
                raise CloudFormatError("lzf: truncated offset")
            ref = op - ((c & 0x1F) << 8) - 1 - src[ip]
            ip += 1
            ln += 2
            if ref < 0 or op + ln > out_len:
                raise CloudFormatError("lzf: back-reference out of range")
            if ref + ln <= op:
                out[op:op + ln] = out[ref:ref + ln]
            else:
                for i in range(ln):
                    out[op + i] = out[ref + i]
            op += ln
    if op != out_len:
        raise CloudFormatError(f"lzf: decoded {op} bytes, header says {out_len}")
    return bytes(out)


def lzf_compress_literal(data: bytes) -> bytes:
    """A valid LZF stream made of literal runs only (test/writer helper; PCL's reader accepts
    any valid stream)."""
    out = bytearray()
    for i in range(0, len(data), 32):
        chunk = data[i:i + 32]
        out.append(len(chunk) - 1)
        out += chunk
    return bytes(out)


# ------------------------------------------------------------------------------------- PCD


@dataclass
class PcdCloud:
    xyz: np.ndarray  # (width*height, 3) float32
    width: int
    height: int
    viewpoint: tuple


def _parse_header(buf: bytes):
    hdr = {}
    pos = 0
    while True:
        nl = buf.find(b"\n", pos)
        if nl < 0:
            raise CloudFormatError("pcd: header not terminated by a DATA line")
        line = buf[pos:nl].decode("ascii", "replace").strip()
        pos = nl + 1
        if not line or line.startswith("#"):
            continue
        key, _, rest = line.partition(" ")
        hdr[key.upper()] = rest.split()
        if key.upper() == "DATA":
            return hdr, pos


def load_pcd_xyz(path: str) -> PcdCloud:
    """pcl::io::loadPCDFile<pcl::PointXYZ>: x, y, z by field name; points = WIDTH*HEIGHT."""
    with open(path, "rb") as f:
        buf = f.read()
    hdr, pos = _parse_header(buf)
    try:
        fields = hdr["FIELDS"]
        sizes = [int(s) for s in hdr["SIZE"]]
        types = hdr["TYPE"]
        counts = [int(c) for c in hdr.get("COUNT", ["1"] * len(fields))]
        width = int(hdr["WIDTH"][0])
        height = int(hdr.get("HEIGHT", ["1"])[0])
        data = hdr["DATA"][0].lower()
    except (KeyError, IndexError, ValueError) as e:
        raise CloudFormatError(f"pcd: bad header ({e})") from None
    if not (len(fields) == len(sizes) == len(types) == len(counts)):
        raise CloudFormatError("pcd: FIELDS/SIZE/TYPE/COUNT lengths differ")
    vp = tuple(float(v) for v in hdr.get("VIEWPOINT", ["0", "0", "0", "1", "0", "0", "0"]))
    npts = width * height
    if "POINTS" in hdr and int(hdr["POINTS"][0]) != npts:
        raise CloudFormatError("pcd: POINTS != WIDTH*HEIGHT")
    for a in "xyz":
        if a not in fields:
            raise CloudFormatError(f"pcd: no field {a}")
    dts = []
    for fl, sz, ty, ct in zip(fields, sizes, types, counts):
        key = (ty.upper(), sz)
        if key not in _PCD_NP:
            raise CloudFormatError(f"pcd: unsupported type {ty}{sz}")
        dts.append((fl if fl != "_" else f"_pad{len(dts)}", _PCD_NP[key], (ct,) if ct > 1 else ()))
    rec = np.dtype(dts)
    xyz = np.empty((npts, 3), dtype=np.float32)
    if data == "ascii":
        tokens = buf[pos:].split()
        ncol = sum(counts)
        if len(tokens) < npts * ncol:
            raise CloudFormatError("pcd: ascii data truncated")
        vals = np.array(tokens[:npts * ncol], dtype=np.float64).reshape(npts, ncol)
        col = 0
        for fl, ct in zip(fields, counts):
            if fl in ("x", "y", "z"):
                xyz[:, "xyz".index(fl)] = vals[:, col]
            col += ct
    elif data == "binary":
        need = npts * rec.itemsize
        if len(buf) - pos < need:
            raise CloudFormatError("pcd: binary data truncated")
        arr = np.frombuffer(buf, dtype=rec, count=npts, offset=pos)
        for i, a in enumerate("xyz"):
            xyz[:, i] = arr[a]
    elif data == "binary_compressed":
        if len(buf) - pos < 8:
            raise CloudFormatError("pcd: compressed header truncated")
        csize, usize = struct.unpack_from("<II", buf, pos)
        raw = lzf_decompress(buf[pos + 8:pos + 8 + csize], usize)
        off = 0  # fields stored one after another (SoA), each npts * size * count bytes
        for fl, sz, ty, ct in zip(fields, sizes, types, counts):
            nb = npts * sz * ct
            if fl in ("x", "y", "z"):
                xyz[:, "xyz".index(fl)] = np.frombuffer(raw, dtype=_PCD_NP[(ty.upper(), sz)],
                                                        count=npts, offset=off)
            off += nb
        if off != usize:
            raise CloudFormatError("pcd: compressed size does not match the fields")
    else:
        raise CloudFormatError(f"pcd: unknown DATA {data}")
    return PcdCloud(xyz, width, height, vp)


def save_pcd_xyz(path: str, xyz: np.ndarray, data: str = "binary") -> None:
    """pcl::PCDWriter::write<PointXYZ>(..., binary=true) layout (app_ros.cpp:172): fields
    x y z, F4, unorganised (HEIGHT 1). `data` may also be "ascii" or "binary_compressed"."""
    P = np.ascontiguousarray(np.asarray(xyz, dtype=np.float32)[:, :3])
    n = len(P)
    head = ("# .PCD v0.7 - Point Cloud Data file format\nVERSION 0.7\nFIELDS x y z\n"
            "SIZE 4 4 4\nTYPE F F F\nCOUNT 1 1 1\n"
            f"WIDTH {n}\nHEIGHT 1\nVIEWPOINT 0 0 0 1 0 0 0\nPOINTS {n}\nDATA {data}\n")
    with open(path, "wb") as f:
        f.write(head.encode("ascii"))
        if data == "binary":
            f.write(P.tobytes())
        elif data == "ascii":
            f.write("".join(f"{x!r} {y!r} {z!r}\n" for x, y, z in P.tolist()).encode("ascii"))
        elif data == "binary_compressed":
            raw = np.ascontiguousarray(P.T).tobytes()
            comp = lzf_compress_literal(raw)
            f.write(struct.pack("<II", len(comp), len(raw)) + comp)
        else:
            raise ValueError(data)


def load_kitti_bin(path: str) -> np.ndarray:
    """KITTI velodyne scan: packed float32 (x, y, z, reflectance) records; the kitti2pcd step
    of bash/kitti2pcd_no_ground.sh keeps x, y, z for PointXYZ."""
    raw = np.fromfile(path, dtype="<f4")
    if raw.size % 4:
        raise CloudFormatError("kitti: size is not a multiple of 16 bytes")
    return np.ascontiguousarray(raw.reshape(-1, 4)[:, :3])


def process_from_file(directory: str):
    """App::processFromFile (app.cpp:250-279): yields (IsometryWithTime, xyz) per recorded
    cloud in pose-file order. A cloud that cannot be read stops the replay, as the reference's
    `return` does (app.cpp:269-272)."""
    for p in read_pose_file(os.path.join(directory, "aicp_input_poses.csv")):
        fn = cloud_file_name(directory, p.counter, p.sec, p.nsec)
        try:
            cloud = load_pcd_xyz(fn)
        except (OSError, CloudFormatError):
            return
        yield p, cloud.xyz


def recorded_sequence_pairs(directory: str, ref_every: int = 5, max_readings: int | None = None):
    """Frame-to-reference pairs from a recorded directory, in App's windowing: the first cloud
    is the first reference (app.cpp:300-313); each later cloud is a reading registered against
    the current reference, and the reference is replaced by the reading that closes every
    `ref_every` readings (reference_update_frequency, app.cpp:383-391; the replacement here is
    the recorded cloud, not the corrected one). Origins are the recorded pose translations
    (octrees_overlap.cpp:184,229-230). Returns dicts in the bench / ResidentBatch layout
    (T_gt = None: recordings carry no ground truth)."""
    pairs = []
    ref = ref_pose = None
    n_read = 0
    for p, xyz in process_from_file(directory):
        if ref is None:
            ref, ref_pose = xyz, p.pose
            continue
        pairs.append(dict(ref=ref, read=xyz, ref_origin=ref_pose[:3, 3].copy(),
                          read_origin=p.pose[:3, 3].copy(), T_gt=None))
        n_read += 1
        if max_readings is not None and n_read >= max_readings:
            break
        if n_read % ref_every == 0:
            ref, ref_pose = xyz, p.pose
    return pairs


def recorded_stream(directory: str, max_readings: int | None = None):
    """The input of App's stream from a recorded directory (processFromFile, app.cpp:250-279): the
    first cloud (first reference), then the readings with their recorded pose translations as
    sensor origins. Returns synthetic.Stream (T_gt entries None: recordings carry no ground
    truth); aicp_hip_sequence_run then builds the references from the corrected readings."""
    from .synthetic import Stream

    first = first_origin = None
    reads, origins = [], []
    for p, xyz in process_from_file(directory):
        if first is None:
            first, first_origin = xyz, p.pose[:3, 3].copy()
            continue
        reads.append(xyz)
        origins.append(p.pose[:3, 3].copy())
        if max_readings is not None and len(reads) >= max_readings:
            break
    if first is None:
        return None
    return Stream(first, first_origin, reads, origins, [None] * len(reads))
