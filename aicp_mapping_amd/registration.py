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
