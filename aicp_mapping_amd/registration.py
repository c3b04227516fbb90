"""Host-side mirror of aicp_core's registration / overlap plugin interfaces over the C-ABI.

Reference interfaces (zbqq/aicp_mapping):
  AbstractRegistrator   aicp_core/include/aicp_registration/abstract_registrator.hpp:8-19
  create_registrator    aicp_core/include/aicp_registration/registration.hpp:9-19
  RegistrationParams    aicp_core/include/aicp_registration/common.hpp:7-23
  AbstractOverlapper    aicp_core/include/aicp_overlap/abstract_overlapper.hpp:13-19
  create_overlapper     aicp_core/include/aicp_overlap/overlap.hpp:9-19
  OverlapParams         aicp_core/include/aicp_overlap/common.hpp:7-14
  App::computeOverlap / computeRegistration / runAicpPipeline
                        aicp_core/src/registration/app.cpp:112-141,187-247

Same method names, argument meaning and error behaviour: clouds are float32 rows of width 3
(packed xyz), 4, 8 or 12 (pcl::PointXYZ / PointXYZRGB / PointXYZRGBNormal, 16 / 32 / 48 B; the
XYZRGBNormal overload is the reference's no-op stub, pointmatcher_registration.cpp:35-44),
transforms 4x4 row-major numpy (Eigen::Matrix4f values), a
ConvergenceError propagates exactly where libpointmatcher's would (uncaught at app.cpp:210),
an unknown registration type prints an error and yields None.
"""
from __future__ import annotations

import abc
import os
import sys
import tempfile
from dataclasses import dataclass, field

import numpy as np

from . import _lib
from ._lib import AICP_RUN_ICP, AICP_RUN_OVERLAP, ConvergenceError, Context  # noqa: F401


@dataclass
class PointmatcherRegistrationParams:
    configFileName: str = ""
    initialTransform: str = ""
    printOutputStatistics: bool = False


@dataclass
class RegistrationParams:
    type: str = ""
    sensorRange: float = -1
    sensorAngularView: float = -1
    loadPosesFrom: str = ""
    initialTransform: str = ""
    pointmatcher: PointmatcherRegistrationParams = field(default_factory=PointmatcherRegistrationParams)


@dataclass
class OctreeOverlapParams:
    # YAMLConfigurator reads it as<float> into a double (yaml_configurator.cpp:81)
    octomapResolution: float = float(np.float32(0.2))


@dataclass
class OverlapParams:
    type: str = ""
    loadPosesFromFile: str = ""
    octree_based: OctreeOverlapParams = field(default_factory=OctreeOverlapParams)


_default_ctx = None


def default_context() -> Context:
    global _default_ctx
    if _default_ctx is None:
        _default_ctx = Context(int(os.environ.get("AICP_HIP_DEVICE", "0")))
    return _default_ctx


class AbstractRegistrator(abc.ABC):
    @abc.abstractmethod
    def registerClouds(self, cloud_ref, cloud_read, final_transform=None): ...

    @abc.abstractmethod
    def getInitializedReading(self): ...

    @abc.abstractmethod
    def getOutputReading(self): ...

    @abc.abstractmethod
    def updateConfigParams(self, config_name: str): ...


class HipRegistration(AbstractRegistrator):
    """PointmatcherRegistration's behaviour (pointmatcher_registration.cpp:14-151) on HIP."""

    def __init__(self, params: RegistrationParams, ctx: Context | None = None):
        self.params_ = params
        self._ctx = ctx
        self.cfg = _lib.default_config()
        self.stats = None
        self._read = None
        self._out = None

    def applyConfig(self):
        path = self.params_.pointmatcher.configFileName
        if not path:
            # icp_.setDefault() uses RandomSampling / SamplingSurfaceNormal: not in this core
            raise _lib.AicpError(_lib.AICP_ERR_UNSUPPORTED, "empty chain file (setDefault) unsupported")
        rc, cfg = _lib.parse_pm_yaml(path)
        if rc == _lib.AICP_ERR_INVALID:
            print(f"[Pointmatcher] Cannot open config file {path}", file=sys.stderr)
            sys.exit(1)
        if rc != _lib.AICP_OK:
            raise _lib.AicpError(rc, f"unsupported chain in {path}")
        self.cfg = cfg

    @property
    def ctx(self) -> Context:  # the HIP context is created on first use
        if self._ctx is None:
            self._ctx = default_context()
        return self._ctx

    def updateConfigParams(self, config_name: str):
        self.params_.pointmatcher.configFileName = config_name

    def registerClouds(self, cloud_ref, cloud_read, final_transform=None):
        """Returns T (4x4); if final_transform (4x4 array) is given it is filled in place.

        PointXYZRGBNormal rows (width 12): the reference's overload is a commented-out stub
        (pointmatcher_registration.cpp:35-44) that leaves final_transform as it is, and so does
        this one (returns final_transform unchanged, None if not given). The C-ABI itself reads
        48-byte rows like any other stride (aicp_pair.ref_stride)."""
        ref = _lib.as_points(cloud_ref)
        read = _lib.as_points(cloud_read)
        if ref.shape[1] == 12 or read.shape[1] == 12:
            return final_transform
        self.applyConfig()
        T, stats, rc = self.ctx.align_batch([dict(ref=ref, read=read)], self.cfg, flags=AICP_RUN_ICP,
                                            raise_on_error=False)
        self.stats = stats[0]
        if rc != _lib.AICP_OK:
            self.ctx.check(rc)
        print(f"[Pointmatcher] Accepted matches (inliers): {self.stats['inlier_ratio'] * 100} %")
        self._read = read
        self._out = None
        self._T = T[0]
        if final_transform is not None:
            final_transform[...] = T[0]
        return T[0]

    def getInitializedReading(self):
        return None if self._read is None else self._read[:, :3].copy()

    def getOutputReading(self):
        if self._out is None and self._read is not None:
            self._out = self.ctx.transform(self._T, self._read)
        return self._out


def create_registrator(parameters: RegistrationParams, ctx: Context | None = None):
    """registration.hpp:9-19 with the HIP core registered as "HIP" (and serving the
    "Pointmatcher" chain files)."""
    if parameters.type in ("HIP", "Pointmatcher"):
        return HipRegistration(parameters, ctx)
    if parameters.type == "GICP":
        return None
    print(f"Invalid registration type {parameters.type}.", file=sys.stderr)
    return None


class AbstractOverlapper(abc.ABC):
    @abc.abstractmethod
    def computeOverlap(self, ref_cloud, read_cloud, ref_pose, read_pose, reading_tree=None): ...

    @abc.abstractmethod
    def getOverlap(self) -> float: ...


class HipOverlapper(AbstractOverlapper):
    """OctreesOverlap::computeOverlap (octrees_overlap.cpp:29-72) as a device voxel-set overlap."""

    def __init__(self, params: OverlapParams, ctx: Context | None = None):
        self.params_ = params
        self.ctx = ctx or default_context()
        self.overlap_ = -1.0
        self.counts = None

    def computeOverlap(self, ref_cloud, read_cloud, ref_pose, read_pose, reading_tree=None):
        """Poses: 4x4 (Eigen::Isometry3d); the sensor origins are their translations.
        Returns None (no octomap tree object is produced)."""
        ro = np.asarray(ref_pose, np.float64)[:3, 3]
        do = np.asarray(read_pose, np.float64)[:3, 3]
        _, stats, rc = self.ctx.align_batch(
            [dict(ref=ref_cloud, read=read_cloud, ref_origin=ro, read_origin=do)],
            flags=AICP_RUN_OVERLAP, resolution=self.params_.octree_based.octomapResolution,
            raise_on_error=True)
        self.overlap_ = float(stats[0]["overlap_percent"])
        self.counts = stats[0]["overlap_keys"]
        return None

    def getOverlap(self) -> float:
        return self.overlap_


def create_overlapper(parameters: OverlapParams, ctx: Context | None = None):
    if parameters.type in ("OctreeBased", "HIP"):
        return HipOverlapper(parameters, ctx)
    return None


def isometry_from_matrix4f(T) -> np.ndarray:
    """fromMatrix4fToIsometry3d (aicp_core/src/utils/common.cpp:4-23): Eigen's Quaternionf of the
    float rotation block (trace branch, else the largest-diagonal branch), cast to double and
    expanded by toRotationMatrix in double; the translation is the float column widened. 4x4
    float64."""
    f = np.float32
    m = np.asarray(T, np.float32).reshape(4, 4)
    q = [f(0)] * 4  # x, y, z, w
    t = f(f(m[0, 0] + m[1, 1]) + m[2, 2])
    if t > f(0):
        t = f(np.sqrt(f(t + f(1))))
        q[3] = f(f(0.5) * t)
        t = f(f(0.5) / t)
        q[0] = f(f(m[2, 1] - m[1, 2]) * t)
        q[1] = f(f(m[0, 2] - m[2, 0]) * t)
        q[2] = f(f(m[1, 0] - m[0, 1]) * t)
    else:
        i = 0
        if m[1, 1] > m[0, 0]:
            i = 1
        if m[2, 2] > m[i, i]:
            i = 2
        j, k = (i + 1) % 3, (i + 2) % 3
        t = f(np.sqrt(f(f(f(m[i, i] - m[j, j]) - m[k, k]) + f(1))))
        q[i] = f(f(0.5) * t)
        t = f(f(0.5) / t)
        q[3] = f(f(m[k, j] - m[j, k]) * t)
        q[j] = f(f(m[j, i] + m[i, j]) * t)
        q[k] = f(f(m[k, i] + m[i, k]) * t)
    x, y, z, w = (float(v) for v in q)
    tx, ty, tz = 2.0 * x, 2.0 * y, 2.0 * z
    twx, twy, twz = tx * w, ty * w, tz * w
    txx, txy, txz = tx * x, ty * x, tz * x
    tyy, tyz, tzz = ty * y, tz * y, tz * z
    out = np.eye(4)
    out[:3, :3] = [[1.0 - (tyy + tzz), txy - twz, txz + twy],
                   [txy + twz, 1.0 - (txx + tzz), tyz - twx],
                   [txz - twy, tyz + twx, 1.0 - (txx + tyy)]]
    out[:3, 3] = m[:3, 3].astype(np.float64)
    return out


class AicpPipeline:
    """The registration hot path of App (app.cpp:112-141, 187-247) for one pair:
    computeOverlap -> ratio auto-tune (clamp + YAML text rewrite) -> registerClouds."""

    def __init__(self, reg_params: RegistrationParams, overlap_params: OverlapParams,
                 registration_config_file: str | None = None, localize_against_prior_map=False,
                 ctx: Context | None = None):
        self.reg_params = reg_params
        self.overlap_params = overlap_params
        self.registr_ = create_registrator(reg_params, ctx)
        self.overlapper_ = create_overlapper(overlap_params, ctx)
        self.registration_config_file = registration_config_file or os.path.join(
            tempfile.gettempdir(), "aicp_hip_icp_autotuned.yaml")
        self.localize_against_prior_map = localize_against_prior_map
        self.octree_overlap_ = -1.0

    def setAndFilterReading(self, raw_reading, prior_pose, working_mode="robot", initialT=None):
        """App::setAndFilterReading (app.cpp:77-99): in "debug" mode the RAW reading is moved by
        initialT_ (pcl::transformPointCloud, float; aicp_hip_transform) and its prior pose becomes
        initialT_ * prior pose, and only then pre-filtered (regionGrowingUniformPlaneSegmentation-
        Filter, aicp_hip_prefilter); "robot" mode pre-filters the reading as given. This is App's
        filter order in debug mode, which aicp_hip_sequence_run (pre-filtered clouds in) does not
        reproduce: the 0.08 m VoxelGrid is world-aligned. Returns (filtered cloud, pose)."""
        from . import filtering

        pose = np.asarray(prior_pose, np.float64)
        cloud = _lib.as_points(raw_reading)[:, :3]
        ctx = self.registr_.ctx if self.registr_ is not None else default_context()
        if working_mode != "robot":
            T = np.eye(4, dtype=np.float32) if initialT is None else np.asarray(initialT, np.float32)
            cloud = ctx.transform(T, cloud)
            pose = isometry_from_matrix4f(T) @ pose  # fromMatrix4fToIsometry3d(initialT_) * reading_pose
        return filtering.regionGrowingUniformPlaneSegmentationFilter(cloud, ctx=ctx), pose

    def computeOverlap(self, ref, read, ref_pose, read_pose):
        if self.localize_against_prior_map:
            self.octree_overlap_ = 50.0
        else:
            self.overlapper_.computeOverlap(ref, read, ref_pose, read_pose)
            self.octree_overlap_ = self.overlapper_.getOverlap()
        return self.octree_overlap_

    def computeRegistration(self, ref, read):
        current_ratio = _lib.autotune_ratio(self.octree_overlap_)  # app.cpp:197-202 (+ text)
        _lib.replace_ratio_config_file(self.reg_params.pointmatcher.configFileName,
                                       self.registration_config_file, current_ratio)
        self.registr_.updateConfigParams(self.registration_config_file)
        return self.registr_.registerClouds(ref, read)

    def runAicpPipeline(self, ref, read, ref_pose, read_pose):
        self.computeOverlap(ref, read, ref_pose, read_pose)
        return self.computeRegistration(ref, read)
