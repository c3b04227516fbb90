"""ctypes binding of libaicp_hip.so (include/aicp_hip.h).

The HIP library is the product: importing this module loads it and raises if it is missing
or does not export the declared entry points. There is no CPU fallback.
"""
from __future__ import annotations

import ctypes as C
import hashlib
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AICP_HIP_LIB") or os.path.join(PKG_DIR, "libaicp_hip.so")  # override: A/B builds

AICP_OK = 0
AICP_ERR_CONVERGENCE = 1
AICP_ERR_INVALID = 2
AICP_ERR_HIP = 3
AICP_ERR_UNSUPPORTED = 4
AICP_ERR_TRANSFORMATION = 5

AICP_RUN_OVERLAP = 1
AICP_RUN_ICP = 2
AICP_RUN_TIME_NN = 4
AICP_SEQ_DEBUG = 8  # aicp_sequence_params.flags: App's "debug" working_mode

EXPORTS = [
    "aicp_hip_create", "aicp_hip_destroy", "aicp_hip_last_error", "aicp_hip_version",
    "aicp_hip_default_config", "aicp_hip_parse_pm_yaml", "aicp_hip_replace_ratio_config_file",
    "aicp_hip_autotune_ratio", "aicp_hip_register", "aicp_hip_register_batch",
    "aicp_hip_overlap", "aicp_hip_overlap_batch", "aicp_hip_align_batch", "aicp_hip_transform", "aicp_hip_crop_box",
    "aicp_hip_batch_upload", "aicp_hip_batch_run", "aicp_hip_batch_free",
    "aicp_hip_last_nn_timing", "aicp_hip_last_phase_ms", "aicp_hip_knn", "aicp_hip_normals",
    "aicp_hip_dists_quantile", "aicp_hip_solve6", "aicp_hip_default_prefilter", "aicp_hip_prefilter",
    "aicp_hip_last_prefilter_stats", "aicp_hip_map_create", "aicp_hip_map_free", "aicp_hip_map_size",
    "aicp_hip_map_download", "aicp_hip_map_crop", "aicp_hip_map_merge", "aicp_hip_map_prefilter",
    "aicp_hip_default_sequence_params", "aicp_hip_sequence_run", "aicp_hip_last_sequence_timing",
    "aicp_hip_map_register_batch", "aicp_hip_multi_create", "aicp_hip_multi_destroy", "aicp_hip_multi_size",
    "aicp_hip_multi_context", "aicp_hip_multi_last_error", "aicp_hip_multi_align_batch",
    "aicp_hip_reference_cache_stats", "aicp_hip_default_options", "aicp_hip_set_options", "aicp_hip_get_options",
    "aicp_hip_test_force_scan_stall", "aicp_hip_sequence_run_raw", "aicp_hip_build_info",
]


_NEWEST = {"aicp_hip_reference_cache_stats", "aicp_hip_default_options", "aicp_hip_set_options",
           "aicp_hip_get_options", "aicp_hip_test_force_scan_stall",
           "aicp_hip_sequence_run_raw", "aicp_hip_build_info"}  # added in r05 / r06


class IcpConfig(C.Structure):
    _fields_ = [
        ("knn_normals", C.c_int32),
        ("nn_epsilon", C.c_float),
        ("nn_max_dist", C.c_float),
        ("trimmed_ratio", C.c_float),
        ("max_iter", C.c_int32),
        ("min_diff_rot", C.c_float),
        ("min_diff_trans", C.c_float),
        ("smooth_length", C.c_int32),
        ("bucket_size", C.c_int32),
        ("knn_match", C.c_int32),
    ]


class IcpStats(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("iterations", C.c_int32),
        ("converged", C.c_int32),
        ("degenerate_normals", C.c_int32),
        ("inlier_ratio", C.c_float),
        ("trimmed_ratio", C.c_float),
        ("overlap_percent", C.c_float),
        ("tree_depth", C.c_int32),
        ("nn_points_touched", C.c_uint64),
        ("nn_nodes_touched", C.c_uint64),
        ("overlap_keys", C.c_uint64 * 3),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k, _ in self._fields_ if k != "overlap_keys"}
        d["overlap_keys"] = [int(x) for x in self.overlap_keys]
        return d


class Pair(C.Structure):
    _fields_ = [
        ("ref", C.POINTER(C.c_float)),
        ("n_ref", C.c_uint64),
        ("ref_stride", C.c_uint64),
        ("read", C.POINTER(C.c_float)),
        ("n_read", C.c_uint64),
        ("read_stride", C.c_uint64),
        ("init_T", C.POINTER(C.c_float)),
        ("ref_origin", C.c_double * 3),
        ("read_origin", C.c_double * 3),
    ]


class PrefilterParams(C.Structure):
    _fields_ = [
        ("leaf_size", C.c_float),
        ("normal_k", C.c_int32),
        ("neighbours", C.c_int32),
        ("min_cluster_size", C.c_int32),
        ("max_cluster_size", C.c_int32),
        ("smoothness_rad", C.c_float),
        ("curvature_threshold", C.c_float),
        ("viewpoint", C.c_float * 3),
    ]


class PrefilterStats(C.Structure):
    _fields_ = [
        ("voxel_ms", C.c_double),
        ("normals_ms", C.c_double),
        ("segment_ms", C.c_double),
        ("device_ms", C.c_double),
        ("wall_ms", C.c_double),
        ("knn_ms", C.c_double),
        ("knn_queries", C.c_uint64),
        ("knn_points_touched", C.c_uint64),
        ("knn_nodes_touched", C.c_uint64),
        ("propagation_passes", C.c_int32),
        ("pad", C.c_int32),
    ]


class Cloud(C.Structure):
    _fields_ = [
        ("pts", C.POINTER(C.c_float)),
        ("n", C.c_uint64),
        ("stride", C.c_uint64),
        ("origin", C.c_double * 3),
    ]


class SequenceParams(C.Structure):
    _fields_ = [
        ("reference_update_frequency", C.c_int32),
        ("max_correction_magnitude", C.c_float),
        ("resolution", C.c_double),
        ("flags", C.c_int32),
    ]


class SequenceResult(C.Structure):
    _fields_ = [
        ("status", C.c_int32),
        ("accepted", C.c_int32),
        ("reference", C.c_int32),
        ("is_reference", C.c_int32),
        ("corrected_origin", C.c_double * 3),
        ("icp", IcpStats),
    ]

    def as_dict(self):
        d = {k: getattr(self, k) for k in ("status", "accepted", "reference", "is_reference")}
        d["corrected_origin"] = [float(x) for x in self.corrected_origin]
        d["icp"] = self.icp.as_dict()
        return d


class Options(C.Structure):
    """aicp_hip_options (include/aicp_hip.h): a context's engine and schedule switches."""
    _fields_ = [
        ("profile", C.c_int32),
        ("nn_engine", C.c_int32),
        ("overlap_path", C.c_int32),
        ("normals_knn_engine", C.c_int32),
        ("select_pair", C.c_int32),
        ("select_fused_from", C.c_int32),
        ("raw_tree_first", C.c_int32),
        ("raw_first_at", C.c_int32),
        ("no_early_exit", C.c_int32),
        ("tree_plan", C.c_int32),
        ("tree_lvl_min", C.c_uint32),
        ("reference_cache", C.c_int32),
        ("oneshot_keep_mib", C.c_uint32),
        ("early_reference", C.c_int32),
        ("read_order_min", C.c_uint64),
    ]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


class SequenceTiming(C.Structure):
    _fields_ = [
        ("windows", C.c_int32),
        ("replans", C.c_int32),
        ("wall_ms", C.c_double),
        ("device_ms", C.c_double),
    ]


def _load():
    if not os.path.exists(LIB_PATH):
        raise ImportError(
            f"{LIB_PATH} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(hipcc --offload-arch=gfx950). There is no CPU fallback.")
    L = C.CDLL(LIB_PATH)
    for name in EXPORTS:
        # (an AICP_HIP_LIB override may be an older build in an A/B run: the newest entry points only)
        if not hasattr(L, name) and not (os.environ.get("AICP_HIP_LIB") and name in _NEWEST):
            raise ImportError(f"{LIB_PATH} does not export {name}")
    vp = C.c_void_p
    fp = C.POINTER(C.c_float)
    dp = C.POINTER(C.c_double)
    ip = C.POINTER(C.c_int32)
    up = C.POINTER(C.c_uint64)
    cfgp = C.POINTER(IcpConfig)
    stp = C.POINTER(IcpStats)
    pp = C.POINTER(Pair)
    sz = C.c_size_t
    L.aicp_hip_create.argtypes = [C.c_int, C.POINTER(vp)]
    L.aicp_hip_destroy.argtypes = [vp]
    L.aicp_hip_destroy.restype = None
    L.aicp_hip_last_error.argtypes = [vp]
    L.aicp_hip_last_error.restype = C.c_char_p
    L.aicp_hip_version.restype = C.c_char_p
    if hasattr(L, "aicp_hip_build_info"):
        L.aicp_hip_build_info.restype = C.c_char_p
    L.aicp_hip_default_config.argtypes = [cfgp]
    L.aicp_hip_default_config.restype = None
    L.aicp_hip_parse_pm_yaml.argtypes = [C.c_char_p, cfgp]
    L.aicp_hip_replace_ratio_config_file.argtypes = [C.c_char_p, C.c_char_p, C.c_float]
    L.aicp_hip_autotune_ratio.argtypes = [C.c_float]
    L.aicp_hip_autotune_ratio.restype = C.c_float
    L.aicp_hip_register.argtypes = [vp, cfgp, pp, fp, stp]
    L.aicp_hip_register_batch.argtypes = [vp, cfgp, pp, sz, fp, stp]
    L.aicp_hip_overlap.argtypes = [vp, pp, C.c_double, fp]
    L.aicp_hip_overlap_batch.argtypes = [vp, pp, sz, C.c_double, fp, stp]
    L.aicp_hip_align_batch.argtypes = [vp, cfgp, pp, sz, C.c_double, C.c_int, fp, stp]
    L.aicp_hip_transform.argtypes = [vp, fp, fp, sz, sz, fp]
    L.aicp_hip_crop_box.argtypes = [vp, fp, sz, sz, C.c_float, C.c_float, fp, fp, C.POINTER(C.c_size_t), fp]
    L.aicp_hip_batch_upload.argtypes = [vp, pp, sz, C.POINTER(vp)]
    L.aicp_hip_batch_run.argtypes = [vp, vp, cfgp, C.c_double, C.c_int, fp, stp]
    L.aicp_hip_batch_free.argtypes = [vp, vp]
    L.aicp_hip_batch_free.restype = None
    L.aicp_hip_last_nn_timing.argtypes = [vp, C.POINTER(C.c_int), dp, dp, up]
    L.aicp_hip_last_phase_ms.argtypes = [vp, dp]
    L.aicp_hip_knn.argtypes = [vp, fp, sz, sz, fp, sz, sz, C.c_int, C.c_float, C.c_float, ip, fp, up]
    L.aicp_hip_normals.argtypes = [vp, fp, sz, sz, C.c_int, fp, ip]
    L.aicp_hip_dists_quantile.argtypes = [vp, fp, sz, C.c_float, fp]
    L.aicp_hip_solve6.argtypes = [vp, dp, dp, dp, ip]
    L.aicp_hip_default_prefilter.argtypes = [C.POINTER(PrefilterParams)]
    L.aicp_hip_default_prefilter.restype = None
    L.aicp_hip_prefilter.argtypes = [vp, C.POINTER(PrefilterParams), fp, sz, sz, fp, C.POINTER(C.c_size_t), fp, ip,
                                     C.POINTER(C.c_size_t), C.POINTER(C.c_size_t)]
    L.aicp_hip_last_prefilter_stats.argtypes = [vp, C.POINTER(PrefilterStats)]
    szp = C.POINTER(C.c_size_t)
    L.aicp_hip_map_create.argtypes = [vp, fp, sz, sz, C.POINTER(vp)]
    L.aicp_hip_map_free.argtypes = [vp, vp]
    L.aicp_hip_map_free.restype = None
    L.aicp_hip_map_size.argtypes = [vp, szp]
    L.aicp_hip_map_download.argtypes = [vp, vp, fp, sz, szp]
    L.aicp_hip_map_crop.argtypes = [vp, vp, C.c_float, C.c_float, fp, fp, sz, szp]
    L.aicp_hip_map_merge.argtypes = [vp, vp, fp, sz, sz, fp]
    L.aicp_hip_map_prefilter.argtypes = [vp, vp, C.POINTER(PrefilterParams)]
    L.aicp_hip_default_sequence_params.argtypes = [C.POINTER(SequenceParams)]
    L.aicp_hip_default_sequence_params.restype = None
    L.aicp_hip_sequence_run.argtypes = [vp, cfgp, C.POINTER(SequenceParams), C.POINTER(Cloud), C.POINTER(Cloud), sz,
                                        fp, C.POINTER(SequenceResult), C.POINTER(C.c_size_t)]
    L.aicp_hip_last_sequence_timing.argtypes = [vp, C.POINTER(SequenceTiming)]
    if hasattr(L, "aicp_hip_sequence_run_raw"):
        L.aicp_hip_sequence_run_raw.argtypes = [vp, cfgp, C.POINTER(SequenceParams), C.POINTER(PrefilterParams),
                                                C.POINTER(Cloud), C.POINTER(Cloud), sz, fp, C.POINTER(SequenceResult),
                                                C.POINTER(C.c_size_t)]
    L.aicp_hip_map_register_batch.argtypes = [vp, cfgp, vp, C.c_float, C.c_float, C.POINTER(Cloud), fp, sz, C.c_int,
                                              fp, stp]
    if hasattr(L, "aicp_hip_reference_cache_stats"):
        L.aicp_hip_reference_cache_stats.argtypes = [vp, C.POINTER(C.c_uint64)]
    if hasattr(L, "aicp_hip_set_options"):
        L.aicp_hip_default_options.argtypes = [C.POINTER(Options)]
        L.aicp_hip_default_options.restype = None
        L.aicp_hip_set_options.argtypes = [vp, C.POINTER(Options)]
        L.aicp_hip_get_options.argtypes = [vp, C.POINTER(Options)]
        L.aicp_hip_test_force_scan_stall.argtypes = [C.c_int]
    L.aicp_hip_multi_create.argtypes = [ip, C.c_int, C.POINTER(vp)]
    L.aicp_hip_multi_destroy.argtypes = [vp]
    L.aicp_hip_multi_destroy.restype = None
    L.aicp_hip_multi_size.argtypes = [vp]
    L.aicp_hip_multi_context.argtypes = [vp, C.c_int]
    L.aicp_hip_multi_context.restype = vp
    L.aicp_hip_multi_last_error.argtypes = [vp]
    L.aicp_hip_multi_last_error.restype = C.c_char_p
    L.aicp_hip_multi_align_batch.argtypes = [vp, cfgp, pp, sz, C.c_double, C.c_int, fp, stp, ip]
    return L


lib = _load()


def build_info() -> str:
    """The loaded library's provenance line (aicp_hip_build_info): "src <hash> arch <gfx> extra
    <flags>", or "" for a library older than the call."""
    return lib.aicp_hip_build_info().decode() if hasattr(lib, "aicp_hip_build_info") else ""


def source_hash(csrc: str = os.path.join(PKG_DIR, "csrc")) -> str:
    """The hash the Makefile embeds: sha256 over its SRCS_HIP, SRCS_CPP and HDRS files and the
    Makefile itself, in that order (first 16 hex digits)."""
    mk = os.path.join(csrc, "Makefile")
    lists = {}
    text = open(mk).read().replace("\\\n", " ")
    for line in text.splitlines():
        for key in ("SRCS_HIP", "SRCS_CPP", "HDRS"):
            if line.startswith(key + " ="):
                lists[key] = line.split("=", 1)[1].split()
    h = hashlib.sha256()
    for f in lists["SRCS_HIP"] + lists["SRCS_CPP"] + lists["HDRS"] + ["Makefile"]:
        with open(os.path.join(csrc, f), "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def provenance() -> dict:
    """Whether the loaded library was built from this tree's sources (bench lines carry it)."""
    info = build_info()
    src = info.split()[1] if info.startswith("src ") else ""
    try:
        tree = source_hash()
    except OSError:
        tree = ""
    return {"library": os.path.abspath(LIB_PATH), "build_info": info, "tree_source_hash": tree,
            "built_from_tree": bool(src) and src == tree}


class AicpError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"aicp_hip error {code}: {msg}")
        self.code = code


class ConvergenceError(AicpError):
    """Maps PM::ConvergenceError (uncaught in the reference, app.cpp:210)."""


class TransformationError(AicpError):
    """Maps PM::TransformationError: RigidTransformation::checkParameters rejected a transform
    applied to the reading (|1 - det R| > 0.001)."""


def default_options(**kw) -> Options:
    """aicp_hip_default_options (the product path) with keyword overrides."""
    o = Options()
    lib.aicp_hip_default_options(C.byref(o))
    for k, v in kw.items():
        if not hasattr(o, k):
            raise AttributeError(f"aicp_hip_options has no field {k}")
        setattr(o, k, v)
    return o


def test_force_scan_stall(on: bool) -> int:
    """aicp_hip_test_force_scan_stall (test hook, the calling thread's device)."""
    return lib.aicp_hip_test_force_scan_stall(1 if on else 0)


def default_config(**kw) -> IcpConfig:
    c = IcpConfig()
    lib.aicp_hip_default_config(C.byref(c))
    for k, v in kw.items():
        setattr(c, k, v)
    return c


def parse_pm_yaml(path: str):
    c = IcpConfig()
    rc = lib.aicp_hip_parse_pm_yaml(path.encode(), C.byref(c))
    return rc, c


def autotune_ratio(overlap_percent: float) -> float:
    return float(lib.aicp_hip_autotune_ratio(overlap_percent))


def replace_ratio_config_file(in_path: str, out_path: str, ratio: float) -> int:
    return lib.aicp_hip_replace_ratio_config_file(in_path.encode(), out_path.encode(), ratio)


def _fptr(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def as_points(p) -> np.ndarray:
    """float32 array of shape (N, W), C-contiguous, xyz in the first 3 floats of each row:
    W = 3 packed, 4 = pcl::PointXYZ (16 B), 8 = PointXYZRGB (32 B), 12 = PointXYZRGBNormal (48 B)
    (the point types of the registerClouds overloads, abstract_registrator.hpp:10-12; the
    XYZRGBNormal overload is a no-op in the reference, see registration.HipRegistration). The
    row stride is passed through the C-ABI, so no copy is made for these layouts."""
    a = np.ascontiguousarray(p, dtype=np.float32)
    if a.ndim != 2 or a.shape[1] not in (3, 4, 8, 12):
        raise ValueError("points must be (N, 3|4|8|12) float32 rows (PointXYZ / XYZRGB / XYZRGBNormal)")
    return a


def make_pair(ref, read, ref_origin=(0, 0, 0), read_origin=(0, 0, 0), init_T=None):
    """Returns (Pair, keepalive). init_T: 4x4 row-major numpy -> column-major float[16]."""
    ref = as_points(ref)
    read = as_points(read)
    keep = [ref, read]
    p = Pair()
    p.ref = _fptr(ref)
    p.n_ref = ref.shape[0]
    p.ref_stride = ref.shape[1] * 4
    p.read = _fptr(read)
    p.n_read = read.shape[0]
    p.read_stride = read.shape[1] * 4
    if init_T is not None:
        t = np.ascontiguousarray(np.asarray(init_T, np.float32).reshape(4, 4).T.reshape(16))
        keep.append(t)
        p.init_T = _fptr(t)
    for k in range(3):
        p.ref_origin[k] = float(ref_origin[k])
        p.read_origin[k] = float(read_origin[k])
    return p, keep


def default_sequence_params(**kw) -> SequenceParams:
    """App's stream settings (aicp_hip_default_sequence_params): reference every 5 accepted
    readings, max_correction_magnitude 1.0, octomap 0.2 m, per-reading overlap auto-tune."""
    p = SequenceParams()
    lib.aicp_hip_default_sequence_params(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def make_cloud(pts, origin=(0, 0, 0)):
    """Returns (Cloud, keepalive) for (N, 3|4|8|12) float32 rows."""
    a = as_points(pts)
    c = Cloud()
    c.pts = _fptr(a)
    c.n = a.shape[0]
    c.stride = a.shape[1] * 4
    for k in range(3):
        c.origin[k] = float(origin[k])
    return c, a


def default_prefilter(**kw) -> PrefilterParams:
    """filteringUtils.cpp:12,22,27-34 (aicp_hip_default_prefilter); keyword overrides."""
    p = PrefilterParams()
    lib.aicp_hip_default_prefilter(C.byref(p))
    for k, v in kw.items():
        if k == "viewpoint":
            for i in range(3):
                p.viewpoint[i] = float(v[i])
        else:
            setattr(p, k, v)
    return p


# aicp_hip_options overrides every new Context starts with (bench.py --opt k=v); empty: the
# library's defaults
CONTEXT_OPTIONS: dict = {}


class Context:
    """One aicp_hip_ctx: a HIP stream + device arena on one GPU."""

    def __init__(self, device: int = 0):
        h = C.c_void_p()
        rc = lib.aicp_hip_create(int(device), C.byref(h))
        if rc != AICP_OK:
            raise AicpError(rc, f"aicp_hip_create(device={device}) failed (no HIP device?)")
        self.h = h
        self.device = device
        if CONTEXT_OPTIONS:
            self.set_options(**CONTEXT_OPTIONS)

    def close(self):
        if getattr(self, "h", None):
            lib.aicp_hip_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def last_error(self) -> str:
        return lib.aicp_hip_last_error(self.h).decode()

    def get_options(self) -> Options:
        o = Options()
        self.check(lib.aicp_hip_get_options(self.h, C.byref(o)))
        return o

    def set_options(self, opt: Options = None, **kw) -> Options:
        """aicp_hip_set_options: `opt` (default: the context's current options) with keyword
        overrides. Returns the options in force before the call."""
        old = self.get_options()
        new = Options.from_buffer_copy(opt if opt is not None else old)
        for k, v in kw.items():
            if not hasattr(new, k):
                raise AttributeError(f"aicp_hip_options has no field {k}")
            setattr(new, k, v)
        self.check(lib.aicp_hip_set_options(self.h, C.byref(new)))
        return old

    def options(self, **kw):
        """with ctx.options(overlap_path=1): ... -- the overrides for the block only."""
        ctx = self

        class _Scope:
            def __enter__(self):
                self.old = ctx.set_options(**kw)
                return ctx

            def __exit__(self, *exc):
                ctx.set_options(self.old)
                return False

        return _Scope()

    def check(self, rc):
        if rc == AICP_ERR_CONVERGENCE:
            raise ConvergenceError(rc, self.last_error())
        if rc == AICP_ERR_TRANSFORMATION:
            raise TransformationError(rc, self.last_error())
        if rc != AICP_OK:
            raise AicpError(rc, self.last_error())

    # -------------------------------------------------------------- batch pipeline ----------
    def align_batch(self, pairs, cfg=None, resolution=0.2, flags=AICP_RUN_ICP, raise_on_error=True):
        """pairs: list of dict(ref, read, ref_origin, read_origin, init_T). Returns (T[n,4,4]
        row-major float32, list of stats dicts, rc)."""
        cfg = cfg or default_config()
        arr = (Pair * len(pairs))()
        keep = []
        for i, pr in enumerate(pairs):
            p, k = make_pair(pr["ref"], pr["read"], pr.get("ref_origin", (0, 0, 0)),
                             pr.get("read_origin", (0, 0, 0)), pr.get("init_T"))
            arr[i] = p
            keep.append(k)
        outT = np.zeros((len(pairs), 16), np.float32)
        st = (IcpStats * len(pairs))()
        rc = lib.aicp_hip_align_batch(self.h, C.byref(cfg), arr, len(pairs), float(resolution),
                                      int(flags), _fptr(outT), st)
        if raise_on_error and rc != AICP_OK:
            self.check(rc)
        T = outT.reshape(-1, 4, 4).transpose(0, 2, 1).copy()
        return T, [s.as_dict() for s in st], rc

    def register(self, ref, read, cfg=None):
        """aicp_hip_register (registerClouds: one pair, identity initial T, the chain's ratio):
        returns (T 4x4 row-major, stats dict)."""
        cfg = cfg or default_config()
        p, keep = make_pair(ref, read)
        outT = np.zeros(16, np.float32)
        st = IcpStats()
        self.check(lib.aicp_hip_register(self.h, C.byref(cfg), C.byref(p), _fptr(outT), C.byref(st)))
        return outT.reshape(4, 4).T.copy(), st.as_dict()

    def overlap(self, ref, read, ref_origin=(0, 0, 0), read_origin=(0, 0, 0), resolution=0.2):
        """aicp_hip_overlap (computeOverlap + getOverlap for one pair): the overlap in percent."""
        p, keep = make_pair(ref, read, ref_origin, read_origin)
        out = np.zeros(1, np.float32)
        self.check(lib.aicp_hip_overlap(self.h, C.byref(p), float(resolution), _fptr(out)))
        return float(out[0])

    def reference_cache_stats(self):
        """aicp_hip_reference_cache_stats: tree hits / builds, overlap-map hits / builds of the
        one-shot calls' resident reference."""
        a = (C.c_uint64 * 4)()
        self.check(lib.aicp_hip_reference_cache_stats(self.h, a))
        return dict(tree_hits=a[0], tree_builds=a[1], ovl_hits=a[2], ovl_builds=a[3])

    def upload(self, pairs):
        return ResidentBatch(self, pairs)

    def sequence_run(self, first, first_origin, readings, origins, cfg=None, params=None, raise_on_error=True,
                     prefilter=None):
        """App's frame-to-reference stream (aicp_hip_sequence_run): the first cloud is the
        reference, readings[i] (prior-pose origin origins[i]) are registered in order with the
        windowed reference update and the max-correction drop. Returns (T[n, 4, 4] row-major
        corrections, list of result dicts, n_done, rc). prefilter (PrefilterParams, or True for
        the defaults): the clouds are RAW and run in App's order (aicp_hip_sequence_run_raw)."""
        cfg = cfg or default_config()
        prm = params or default_sequence_params()
        if prefilter is True:
            prefilter = default_prefilter()
        n = len(readings)
        fc, keep0 = make_cloud(first, first_origin)
        arr = (Cloud * max(n, 1))()
        keep = [keep0]
        for i, r in enumerate(readings):
            c, k = make_cloud(r, origins[i])
            arr[i] = c
            keep.append(k)
        outT = np.zeros((max(n, 1), 16), np.float32)
        res = (SequenceResult * max(n, 1))()
        done = C.c_size_t(0)
        if prefilter is not None:
            rc = lib.aicp_hip_sequence_run_raw(self.h, C.byref(cfg), C.byref(prm), C.byref(prefilter), C.byref(fc), arr,
                                               n, _fptr(outT), res, C.byref(done))
        else:
            rc = lib.aicp_hip_sequence_run(self.h, C.byref(cfg), C.byref(prm), C.byref(fc), arr, n, _fptr(outT), res,
                                           C.byref(done))
        if raise_on_error and rc != AICP_OK:
            self.check(rc)
        T = outT[:n].reshape(-1, 4, 4).transpose(0, 2, 1).copy()
        return T, [res[i].as_dict() for i in range(done.value)], done.value, rc

    def last_sequence_timing(self):
        t = SequenceTiming()
        self.check(lib.aicp_hip_last_sequence_timing(self.h, C.byref(t)))
        return {k: getattr(t, k) for k, _ in SequenceTiming._fields_}

    def last_nn_timing(self):
        n = C.c_int()
        ms = C.c_double()
        by = C.c_double()
        q = C.c_uint64()
        lib.aicp_hip_last_nn_timing(self.h, C.byref(n), C.byref(ms), C.byref(by), C.byref(q))
        return dict(launches=n.value, total_ms=ms.value, bytes=by.value, queries=q.value)

    def last_phase_ms(self):
        a = (C.c_double * 5)()
        lib.aicp_hip_last_phase_ms(self.h, a)
        return dict(overlap=a[0], normals=a[1], matcher_tree=a[2], icp_loop=a[3], total=a[4])

    # -------------------------------------------------------------- kernel-level -----------
    def knn(self, pts, queries, k=1, eps=0.0, max_dist=float("inf")):
        pts = as_points(pts)
        q = as_points(queries)
        ids = np.zeros((q.shape[0], k), np.int32)
        d2 = np.zeros((q.shape[0], k), np.float32)
        touched = np.zeros(2, np.uint64)
        rc = lib.aicp_hip_knn(self.h, _fptr(pts), pts.shape[0], pts.shape[1] * 4, _fptr(q), q.shape[0],
                              q.shape[1] * 4, int(k), float(eps), float(max_dist),
                              ids.ctypes.data_as(C.POINTER(C.c_int32)), _fptr(d2),
                              touched.ctypes.data_as(C.POINTER(C.c_uint64)))
        self.check(rc)
        return ids, d2, int(touched[0]), int(touched[1])

    def normals(self, pts, knn=20):
        pts = as_points(pts)
        out = np.zeros((pts.shape[0], 3), np.float32)
        deg = C.c_int32()
        rc = lib.aicp_hip_normals(self.h, _fptr(pts), pts.shape[0], pts.shape[1] * 4, int(knn), _fptr(out),
                                  C.byref(deg))
        self.check(rc)
        return out, deg.value

    def dists_quantile(self, d2, quantile):
        d2 = np.ascontiguousarray(d2, np.float32).ravel()
        out = C.c_float()
        rc = lib.aicp_hip_dists_quantile(self.h, _fptr(d2), d2.size, float(quantile), C.byref(out))
        self.check(rc)
        return out.value

    def solve6(self, A, b):
        A = np.ascontiguousarray(A, np.float64).reshape(36)
        b = np.ascontiguousarray(b, np.float64).reshape(6)
        x = np.zeros(6, np.float64)
        path = C.c_int32()
        dp = C.POINTER(C.c_double)
        rc = lib.aicp_hip_solve6(self.h, A.ctypes.data_as(dp), b.ctypes.data_as(dp), x.ctypes.data_as(dp),
                                 C.byref(path))
        self.check(rc)
        return x, path.value

    def transform(self, T, pts):
        pts = as_points(pts)
        t = np.ascontiguousarray(np.asarray(T, np.float32).reshape(4, 4).T.reshape(16))
        out = np.zeros((pts.shape[0], 3), np.float32)
        rc = lib.aicp_hip_transform(self.h, _fptr(t), _fptr(pts), pts.shape[0], pts.shape[1] * 4, _fptr(out))
        self.check(rc)
        return out

    def crop_box(self, pts, mn, mx, origin):
        """getPointsInOrientedBox (filteringUtils.cpp:619-637) on device: returns (kept xyz in
        input order, box angles rx, ry, rz). origin is a 4x4 row-major pose (Matrix4f values)."""
        pts = as_points(pts)
        o = np.ascontiguousarray(np.asarray(origin, np.float32).reshape(4, 4).T.reshape(16))
        out = np.zeros((pts.shape[0], 3), np.float32)
        m = C.c_size_t(0)
        rpy = np.zeros(3, np.float32)
        rc = lib.aicp_hip_crop_box(self.h, _fptr(pts), pts.shape[0], pts.shape[1] * 4, mn, mx, _fptr(o),
                                   _fptr(out), C.byref(m), _fptr(rpy))
        self.check(rc)
        return out[:m.value].copy(), rpy

    def last_prefilter_stats(self):
        st = PrefilterStats()
        self.check(lib.aicp_hip_last_prefilter_stats(self.h, C.byref(st)))
        return {k: getattr(st, k) for k, _ in PrefilterStats._fields_ if k != "pad"}

    def prefilter(self, pts, params=None, details=False):
        """regionGrowingUniformPlaneSegmentationFilter (filteringUtils.cpp:5-45) on device.
        Returns the kept points (clusters concatenated), or with details=True a dict with
        out, sampled (V, 8) {x, y, z, curvature, nx, ny, nz, 0}, labels (V,) and n_clusters."""
        pts = as_points(pts)
        n = pts.shape[0]
        prm = params or default_prefilter()
        out = np.zeros((max(n, 1), 3), np.float32)
        m, ns, nc = C.c_size_t(0), C.c_size_t(0), C.c_size_t(0)
        sampled = np.zeros((max(n, 1), 8), np.float32) if details else None
        labels = np.zeros(max(n, 1), np.int32) if details else None
        rc = lib.aicp_hip_prefilter(self.h, C.byref(prm), _fptr(pts), n, pts.shape[1] * 4, _fptr(out), C.byref(m),
                                    _fptr(sampled) if details else None,
                                    labels.ctypes.data_as(C.POINTER(C.c_int32)) if details else None,
                                    C.byref(ns), C.byref(nc))
        self.check(rc)
        if not details:
            return out[:m.value].copy()
        V = ns.value
        return dict(out=out[:m.value].copy(), sampled=sampled[:V].copy(), labels=labels[:V].copy(),
                    n_clusters=nc.value)


class ResidentBatch:
    """Pairs uploaded once to HBM (aicp_hip_batch_upload), run many times."""

    def __init__(self, ctx: Context, pairs):
        self.ctx = ctx
        self.n = len(pairs)
        arr = (Pair * self.n)()
        keep = []
        for i, pr in enumerate(pairs):
            p, k = make_pair(pr["ref"], pr["read"], pr.get("ref_origin", (0, 0, 0)),
                             pr.get("read_origin", (0, 0, 0)), pr.get("init_T"))
            arr[i] = p
            keep.append(k)
        h = C.c_void_p()
        rc = lib.aicp_hip_batch_upload(ctx.h, arr, self.n, C.byref(h))
        ctx.check(rc)
        self.h = h
        self.outT = np.zeros((self.n, 16), np.float32)
        self.stats = (IcpStats * self.n)()

    def run(self, cfg=None, resolution=0.2, flags=AICP_RUN_ICP | AICP_RUN_OVERLAP, raise_on_error=True):
        cfg = cfg or default_config()
        rc = lib.aicp_hip_batch_run(self.ctx.h, self.h, C.byref(cfg), float(resolution), int(flags),
                                    _fptr(self.outT), self.stats)
        if raise_on_error and rc != AICP_OK:
            self.ctx.check(rc)
        return rc

    def transforms(self):
        return self.outT.reshape(-1, 4, 4).transpose(0, 2, 1).copy()

    def stats_dicts(self):
        return [s.as_dict() for s in self.stats]

    def free(self):
        if getattr(self, "h", None):
            lib.aicp_hip_batch_free(self.ctx.h, self.h)
            self.h = None

    def __del__(self):
        self.free()


class MultiContext:
    """aicp_hip_multi: one context and host thread per device for independent pairs;
    the C++ host's form of the torch.distributed path in bench.py. `devices` may repeat a device."""

    def __init__(self, devices=None, n_devices: int = 0):
        h = C.c_void_p()
        if devices is not None:
            arr = (C.c_int * len(devices))(*[int(d) for d in devices])
            rc = lib.aicp_hip_multi_create(arr, len(devices), C.byref(h))
        else:
            rc = lib.aicp_hip_multi_create(None, int(n_devices), C.byref(h))
        if rc != AICP_OK:
            raise AicpError(rc, f"aicp_hip_multi_create(devices={devices}, n={n_devices}) failed")
        self.h = h

    def size(self) -> int:
        return lib.aicp_hip_multi_size(self.h)

    def close(self):
        if getattr(self, "h", None):
            lib.aicp_hip_multi_destroy(self.h)
            self.h = None

    def __del__(self):
        self.close()

    def align_batch(self, pairs, cfg=None, resolution=0.2, flags=AICP_RUN_ICP, raise_on_error=True):
        """Context.align_batch over the devices. Returns (T[n,4,4] row-major, stats dicts, the
        device of each pair, rc)."""
        cfg = cfg or default_config()
        arr = (Pair * len(pairs))()
        keep = []
        for i, pr in enumerate(pairs):
            p, k = make_pair(pr["ref"], pr["read"], pr.get("ref_origin", (0, 0, 0)),
                             pr.get("read_origin", (0, 0, 0)), pr.get("init_T"))
            arr[i] = p
            keep.append(k)
        outT = np.zeros((len(pairs), 16), np.float32)
        st = (IcpStats * len(pairs))()
        dev = np.zeros(len(pairs), np.int32)
        rc = lib.aicp_hip_multi_align_batch(self.h, C.byref(cfg), arr, len(pairs), float(resolution), int(flags),
                                            _fptr(outT), st, dev.ctypes.data_as(C.POINTER(C.c_int)))
        if raise_on_error and rc != AICP_OK:
            raise AicpError(rc, lib.aicp_hip_multi_last_error(self.h).decode())
        T = outT.reshape(-1, 4, 4).transpose(0, 2, 1).copy()
        return T, [s.as_dict() for s in st], dev, rc
