"""The C++ drop-in shim (integration/hip_registration.hpp) against the reference interfaces.

HipRegistration / HipOverlapper implement aicp::AbstractRegistrator / AbstractOverlapper
(abstract_registrator.hpp:8-19, abstract_overlapper.hpp:13-19). PCL, Eigen and octomap are not in
this image, so tests/shim/stubs restates the two interfaces and stands in for the point / matrix
types; tests/shim/shim_main.cpp drives the shims through the factories the way App does and calls
libaicp_hip.so through include/aicp_hip.h.
"""
import os
import shutil
import subprocess

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
SHIM = os.path.join(HERE, "shim")
CHAIN = os.path.join(HERE, "golden", "icp_autotuned_default.yaml")
LIB = os.path.join(ROOT, "aicp_mapping_amd", "libaicp_hip.so")


def _compile(out):
    cmd = ["g++", "-std=c++14", "-Wall", "-Wextra", "-Werror", "-O1", "-I", os.path.join(SHIM, "stubs"),
           "-I", os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "integration"),
           os.path.join(SHIM, "shim_main.cpp"), "-o", out, "-L", os.path.dirname(LIB), "-laicp_hip",
           "-Wl,-rpath," + os.path.dirname(LIB), "-Wl,-rpath-link,/opt/rocm/lib"]
    r = subprocess.run(cmd, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr


@pytest.mark.skipif(shutil.which("g++") is None or not os.path.exists(LIB), reason="needs g++ and libaicp_hip.so")
def test_shim_compiles_and_behaves_without_device(tmp_path):
    """Compiles with -Wall -Wextra -Werror against the restated interfaces (every pure virtual
    overridden, computeOverlap's poses by value), the factories create the HIP types, an unknown
    type gives nullptr, an empty chain is refused, XYZRGBNormal is a no-op and the chain parses."""
    exe = str(tmp_path / "shim_main")
    _compile(exe)
    r = subprocess.run([exe, "cpu", CHAIN], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "cpu ok: knn 20 eps 3.16 ratio 0.70 maxIter 20" in r.stdout
    assert "Invalid registration type Nope." in r.stderr


@pytest.mark.gpu
def test_shim_registers_like_the_c_abi(tmp_path, oracle):
    """The prebuilt shim binary (tests/shim/shim_main, built by __graft_entry__.build) registers a
    pair through AbstractRegistrator and AbstractOverlapper: T equals the C-ABI's bit for bit,
    the XYZRGB overload gives the same T, and the overlap equals the oracle's."""
    import aicp_mapping_amd._lib as L
    from aicp_mapping_amd import synthetic as sy

    exe = os.path.join(SHIM, "shim_main")
    assert os.path.exists(exe), "tests/shim/shim_main missing: run __graft_entry__.build()"
    pr = sy.make_pair(9000, 9000, seed=41)
    pr.ref.astype(np.float32).tofile(tmp_path / "ref.bin")
    pr.read.astype(np.float32).tofile(tmp_path / "read.bin")
    args = [exe, "gpu", CHAIN, str(tmp_path / "ref.bin"), str(tmp_path / "read.bin")]
    args += ["%.17g" % v for v in pr.ref_origin] + ["%.17g" % v for v in pr.read_origin]
    r = subprocess.run(args, capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stdout + r.stderr
    lines = {ln.split()[0]: ln.split()[1:] for ln in r.stdout.splitlines() if ln and ln.split()[0] in
             ("T", "T_rgb", "overlap", "out")}
    T = np.array([np.float32(x) for x in lines["T"]], np.float32).reshape(4, 4).T
    T_rgb = np.array([np.float32(x) for x in lines["T_rgb"]], np.float32).reshape(4, 4).T
    ctx = L.Context(0)
    Tc, st, rc = ctx.align_batch([dict(ref=pr.ref, read=pr.read)], L.default_config(), flags=L.AICP_RUN_ICP)
    ctx.close()
    assert rc == 0
    np.testing.assert_array_equal(T, Tc[0])
    np.testing.assert_array_equal(T_rgb, Tc[0])
    ov, _ = oracle.overlap(pr.ref, pr.ref_origin, pr.read, pr.read_origin, float(np.float32(0.2)))
    assert np.float32(lines["overlap"][0]) == np.float32(ov)
    assert int(lines["out"][0]) == len(pr.read)
    rc1, T1, _ = oracle.icp(pr.ref, pr.read, oracle.default_config(trimmed_ratio=0.7))
    rr, tt = sy.rot_err(T1, T)
    assert rc1 == 0 and rr <= 1e-4 and tt <= 1e-3
