#!/usr/bin/env python3
"""Benchmark: aligned clouds/s (+ ICP iterations/s) on the BASELINE.json workloads.

Default (C2): App's frame-to-reference stream (app.cpp:282-414) of an ANYmal VLP-16 batch_size=80
accumulation: a first cloud, then 64 readings of N = 120 000 points, each registered against the
current reference (octree overlap -> auto-tuned trimmed ratio -> ICP), the reference rebuilt from
every 5th accepted reading corrected by its own T (the dependency chain of the reference). A
step = one aicp_hip_sequence_run over the 64 host clouds: H2D, every device phase and the read-back
of T are inside the timed region (§8(d): host xyz in -> T out). Each rank runs its own stream
(weak scaling); RCCL all-gathers the per-reading {T, iterations, inlier ratio}.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--config c2|c3|c4|c5|single|app|prefilter]
    torchrun --nproc-per-node N bench.py --gpus N ...

Other configs: c3 (KITTI HDL-64 stream, N = 600 000), c4 (localization against a resident
1 M-point map, device crops as references, r = 0.5), c5 (1024 independent pairs of 60 000 points
sharded i mod G), single (one C2 pair through aicp_hip_register, latency), app (the C2 readings
through App's per-reading calls, overlap + registerClouds, with the reference cache), prefilter
(§8(f) rank 2). The line carries the NN kernel's roofline (HIP events on its stream), the oracle as
cpu_baseline (median of 5 bounded samples on this host) and parity against it.
"""
from __future__ import annotations

import argparse
import json
import os
import platform
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def make_raw_clouds(n_clouds, half, spacing, seed):
    """Raw (pre-filter) clouds of the C2 setting: an 80-scan VLP-16 batch accumulation over the
    synthetic scene, ~2.4 M points at the defaults, one per sensor position along x."""
    from aicp_mapping_amd import synthetic as sy

    scene = sy.make_scene(seed)
    out = []
    for i in range(n_clouds):
        rng = np.random.default_rng(seed * 1000 + i)
        out.append(sy.sample_scene(scene, rng, np.array([0.3 * i, 0.0, 0.7]), half=half,
                                   spacing=spacing).astype(np.float32))
    return out


def bench_prefilter(args):
    """regionGrowingUniformPlaneSegmentationFilter (filteringUtils.cpp:5-45) per raw cloud on one
    GPU per rank (clouds are independent: replicas, weak scaling). value = clouds / device time
    (input uploaded -> clusters ready); the PCIe- and host-packing-inclusive rate is reported
    beside it (the C-ABI takes host buffers like the PCL call)."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")
    import aicp_mapping_amd._lib as L
    from aicp_mapping_amd import sharding as sh

    n_clouds = max(1, min(args.steps, 4))
    clouds = make_raw_clouds(n_clouds, 25.0, 0.035, seed=1 + rank)
    ctx = L.Context(local_rank)
    for i in range(args.warmup):
        ctx.prefilter(clouds[i % n_clouds])
    if dist is not None:
        import torch

        torch.cuda.synchronize()
        dist.barrier()
    dev_ms = wall_ms = knn_ms = knn_bytes = 0.0
    kept = sampled = 0
    outs = []
    t0 = time.perf_counter()
    for i in range(args.steps):
        o = ctx.prefilter(clouds[i % n_clouds])
        st = ctx.last_prefilter_stats()
        dev_ms += st["device_ms"]
        wall_ms += st["wall_ms"]
        knn_ms += st["knn_ms"]
        knn_bytes += st["knn_queries"] * (16 + 4 * 30) + 16 * (st["knn_points_touched"] + st["knn_nodes_touched"])
        kept += len(o)
        sampled += st["knn_queries"]
        if i < n_clouds:
            outs.append(o)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = sh.max_over_ranks(elapsed, dist, device="cuda")
        dev_ms = sh.max_over_ranks(dev_ms, dist, device="cuda")
    if rank == 0:
        n_in = int(np.mean([len(c) for c in clouds]))
        achieved = knn_bytes / (knn_ms * 1e-3) / 1e9
        out = {
            "metric": "prefiltered_clouds_per_s (regionGrowingUniformPlaneSegmentationFilter per raw cloud)",
            "value": round(world * args.steps / (dev_ms * 1e-3), 3),
            "unit": "clouds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(dev_ms / args.steps, 3),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f32 (PCL float arithmetic; computeRoots' atan2/cos/sin in f64 rounded to f32)",
            "data": "synthetic raw clouds (seeded planar scene, 0.035 m spacing, 0.01 m noise)",
            "config": {"workload": "pre-filter of C2 raw clouds: %d distinct clouds of ~%d points (+-25 m), "
                                   "VoxelGrid 0.08 -> NormalEstimation k30 -> RegionGrowing (min 50, 15 nbrs, "
                                   "3 deg, curvature 1.0)" % (n_clouds, n_in),
                       "parallelism": "independent clouds per rank (replicas)"},
            "points_in_per_cloud": n_in,
            "sampled_per_cloud": round(sampled / args.steps),
            "kept_per_cloud": round(kept / args.steps),
            "wall_ms_per_cloud_incl_pcie": round(wall_ms / args.steps, 3),
            "clouds_per_s_incl_pcie": round(args.steps / (wall_ms * 1e-3), 3),
            "timed_loop_ms_per_cloud": round(1e3 * elapsed / args.steps, 3),
            "phase_ms_per_cloud": {k: round(v, 3) for k, v in zip(
                ["voxel_grid", "tree_knn_normals", "region_growing_extract"],
                [st["voxel_ms"], st["normals_ms"], st["segment_ms"]])},
            "propagation_passes": st["propagation_passes"],
            "roofline": {
                "kernel": "k_knn_ids<30> (exact libnabo kNN-30 of every sampled point, LDS far frames)",
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": None,
                "avg_launch_us": round(1e3 * knn_ms / args.steps, 2),
                "algorithmic_bytes_per_launch": round(knn_bytes / args.steps),
                "bytes_model": "Q*(16 + 4*30) + 16*(touched points + touched nodes)",
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle as po

            po.lib()
            done, same = 0, 0
            t1 = time.perf_counter()
            for i, c in enumerate(clouds):
                r = po.prefilter(c)
                done += 1
                same += int(np.array_equal(r["out"], outs[i]))
                if time.perf_counter() - t1 > args.cpu_budget:
                    break
            dt = time.perf_counter() - t1
            out["cpu_baseline"] = {"value": done / dt, "unit": "clouds/s", "cores": 1, "kind": "port",
                                   "sample": f"first {done} of the {n_clouds} clouds (~{n_in} points each), oracle "
                                             f"restatement of the PCL chain on 1 host core ({cpu_model()}); "
                                             f"{dt:.1f} s"}
            out["parity_vs_oracle"] = {"clouds": done, "bit_exact_outputs": same}
        print(json.dumps(out))
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def _stream_reading(a):
    from aicp_mapping_amd import synthetic as sy

    seed, i, n = a
    return sy.stream_reading(seed, i, n)


def make_stream(n_readings, n_points, seed):
    """synthetic.make_stream built in a process pool (16 workers: the box's CPU share)."""
    from concurrent.futures import ProcessPoolExecutor

    from aicp_mapping_amd import synthetic as sy

    first, o0 = sy.stream_first(seed, n_points)
    with ProcessPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        out = list(ex.map(_stream_reading, [(seed, i, n_points) for i in range(n_readings)]))
    return sy.Stream(first, o0, [r[0] for r in out], [r[1] for r in out], [r[2] for r in out])


def _c5_pair(seed_points):
    from aicp_mapping_amd import synthetic as sy

    seed, n = seed_points
    pr = sy.make_pair(n, n, seed=seed)
    return dict(ref=pr.ref, read=pr.read, ref_origin=pr.ref_origin, read_origin=pr.read_origin, T_gt=pr.T_gt)


def make_c5_pairs(n_total, n_points, rank, world):
    """C5: independent pairs, seeds 1000..; rank g takes pairs i = g mod G."""
    from concurrent.futures import ProcessPoolExecutor

    from aicp_mapping_amd import sharding as sh

    mine = sh.shard_pairs(n_total, world, rank)
    with ProcessPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        return list(ex.map(_c5_pair, [(1000 + i, n_points) for i in mine], chunksize=4))


def _c4_reading(a):
    from aicp_mapping_amd import synthetic as sy

    seed, i, n = a
    read, origin, Tg = sy.stream_reading(seed, i, n)
    Ti = np.linalg.inv(Tg)
    pose = Ti @ sy.make_T(yaw_deg=0.0, pitch_deg=0.0, roll_deg=0.0, t=((i + 1) * 0.3, 0.0, 0.7))
    return read, pose, Tg


def make_c4(n_readings, n_points, map_points, seed):
    """C4 localization-only: a resident map of map_points over the whole scene and
    a stream of VLP-16 readings with their prior poses (drifted odometry)."""
    from concurrent.futures import ProcessPoolExecutor

    from aicp_mapping_amd import synthetic as sy

    scene = sy.make_scene(seed)
    rng = np.random.default_rng(seed * 7919 + 77)
    mp = sy.sample_scene(scene, rng, np.array([0.0, 0.0, 0.7]), half=40.0)
    if len(mp) > map_points:
        mp = mp[rng.choice(len(mp), size=map_points, replace=False)]
    with ProcessPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        out = list(ex.map(_c4_reading, [(seed, i, n_points) for i in range(n_readings)]))
    return mp.astype(np.float32), [o[0] for o in out], [o[1] for o in out], [o[2] for o in out]


def init_dist():
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch
        import torch.distributed as dist

        torch.cuda.set_device(local_rank)
        dist.init_process_group(backend="nccl")
    return rank, world, local_rank, dist


def sync(dist):
    if dist is not None:
        import torch

        torch.cuda.synchronize()
        dist.barrier()


def median_rate(fn, reps):
    """fn() -> (units, seconds) per repetition; the median rate and the per-rep rates."""
    rates = []
    for _ in range(reps):
        u, dt = fn()
        rates.append(u / dt)
    return float(np.median(rates)), rates


def roofline_nn(t, kernel):
    """roofline object of the NN kernel from aicp_hip_last_nn_timing sums (HIP events recorded
    on the stream the NN kernel runs on)."""
    n = max(1, t["launches"])
    avg_ms = t["total_ms"] / n
    achieved = (t["bytes"] / n) / (avg_ms * 1e-3) / 1e9 if t["launches"] else 0.0
    return {
        "kernel": kernel,
        "bound": "hbm",
        "achieved": round(achieved, 1),
        "peak": HBM_PEAK_GBS,
        "unit": "GB/s",
        "frac": round(achieved / HBM_PEAK_GBS, 4),
        "traffic": None,
        "avg_launch_us": round(1e3 * avg_ms, 2),
        "launches": t["launches"],
        "algorithmic_bytes_per_launch": round(t["bytes"] / n),
        "bytes_model": "N*(12+8) + V*16 + W*8 (SURVEY §8(d)); V, W = touched points / inner nodes",
    }


def load_traffic(name):
    """PMC traffic (HBM bytes per NN launch) committed under profiles/ from a separate rocprofv3
    --pmc pass of the same workload (tools/profile.sh); None when absent."""
    path = os.path.join(ROOT, "profiles", name)
    try:
        return json.load(open(path))
    except (OSError, ValueError):
        return None


def add_traffic(rf, name):
    """PMC HBM bytes per launch (profiles/<name>, tools/profile.sh) into the roofline object, and
    the fraction of peak they are at this run's launch time beside the algorithmic fraction (on
    the C2 window the tree and the points stay in L2 / MALL, so the counters see far fewer bytes
    than the algorithmic model counts)."""
    tr = load_traffic(name)
    if not tr or not tr.get("bytes_per_launch") or not rf.get("avg_launch_us"):
        return
    rf["traffic"] = tr["bytes_per_launch"]
    rf["traffic_source"] = tr.get("source", name)
    rf["traffic_frac"] = round(tr["bytes_per_launch"] / (rf["avg_launch_us"] * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)


def base_line(args, world, metric, value, unit, ms_per_step, dtype, data, config, scaling="weak", hib=True):
    import aicp_mapping_amd._lib as L

    return {
        "metric": metric,
        "value": round(value, 3),
        "unit": unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 3),
        "higher_is_better": hib,
        "scaling": scaling,
        "vs_baseline": None,
        "dtype": dtype,
        "data": data,
        "config": config,
        # the library this line measured and whether it was built from this tree's sources
        # (aicp_hip_build_info against the sources' hash)
        "build": L.provenance(),
    }


METRIC = "aligned_clouds_per_s (ICP iterations/sec + aligned clouds/sec, 80-scan VLP-16 batch)"
DTYPE = "f32 (point arithmetic; 6x6/3x3 reductions and solves in f64)"
DATA = "synthetic (seeded planar scene per SURVEY §8(d); no recordings in the reference)"
CHAIN = ("icp_autotuned_default.yaml (SurfaceNormal knn20, KDTree knn1 eps3.16, TrimmedDist auto-tuned, "
         "PointToPlane, Counter20 + Differential)")


def bench_stream(args):
    """C2 / C3: App's frame-to-reference stream, host clouds in -> corrections out."""
    import aicp_mapping_amd._lib as L
    from aicp_mapping_amd import sharding as sh
    from aicp_mapping_amd import synthetic as sy

    rank, world, local_rank, dist = init_dist()
    if args.data:  # a recording in the reference's offline layout (§8(f) rank 3)
        from aicp_mapping_amd import cloud_io

        st = cloud_io.recorded_stream(args.data, args.pairs)
        if st is None or not st.readings:
            raise SystemExit(f"--data {args.data}: no readable pose/cloud pairs")
        n_read = len(st.readings)
        n_pts = int(np.mean([len(r) for r in st.readings]))
    else:
        n_read = args.pairs or 64
        n_pts = args.points or (120000 if args.config == "c2" else 600000)
        st = make_stream(n_read, n_pts, seed=1 + rank)
    ctx = L.Context(local_rank)
    cfg = L.default_config()
    debug = args.working_mode == "debug"
    flags = L.AICP_RUN_OVERLAP | (L.AICP_SEQ_DEBUG if debug else 0)
    prm = L.default_sequence_params(reference_update_frequency=args.ref_every, flags=flags)
    # HIP events on the NN launches (AICP_RUN_TIME_NN) only in the last timed step: each timed
    # launch costs ~11 us of dispatch gaps around the NN on the ICP stream (r04 kernel trace:
    # update -> NN 7 us, NN -> select 4.5 us, against ~0 between the other kernels), ~5 % of a
    # C2 window, so the roofline's launch average comes from one step of the timed region
    prm_t = L.default_sequence_params(reference_update_frequency=args.ref_every, flags=flags | L.AICP_RUN_TIME_NN)

    def step(timed=False):
        T, out, done, rc = ctx.sequence_run(st.first, st.first_origin, st.readings, st.origins, cfg,
                                            prm_t if timed else prm, prefilter=True if args.raw else None)
        if dist is not None:
            sh.gather_records(sh.pack_records(T.transpose(0, 2, 1).reshape(-1, 16),
                                              [o["icp"]["iterations"] for o in out],
                                              [o["icp"]["inlier_ratio"] for o in out]), dist, device="cuda")
        return T, out

    for _ in range(args.warmup):
        step()
    sync(dist)
    nn = dict(launches=0, total_ms=0.0, bytes=0.0)
    iters = 0
    dev_ms = wall_ms = 0.0
    windows = replans = 0
    t0 = time.perf_counter()
    for k_step in range(args.steps):
        T, out = step(timed=k_step == args.steps - 1)
        t = ctx.last_nn_timing()
        if t["launches"]:  # (the algorithmic bytes come with every step; the timing with the last)
            for k in ("launches", "total_ms", "bytes"):
                nn[k] += t[k]
        iters += sum(o["icp"]["iterations"] for o in out)
        tm = ctx.last_sequence_timing()
        dev_ms += tm["device_ms"]
        wall_ms += tm["wall_ms"]
        windows, replans = tm["windows"], tm["replans"]
    sync(dist)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = sh.max_over_ranks(elapsed, dist, device="cuda")
        iters = int(sh.sum_over_ranks(float(iters), dist, device="cuda"))
    # the same readings as a batch of independent pairs (r02's workload shape): reading i against
    # the first cloud (i < 5) or the UNcorrected reading 5*(i//5)-1, uploaded once, run resident
    batched = None
    if rank == 0 and not args.no_batched:
        refs = [(st.first, st.first_origin)] + [(st.readings[j], st.origins[j]) for j in range(4, n_read, 5)]
        pairs = [dict(ref=refs[i // 5][0], read=st.readings[i], ref_origin=refs[i // 5][1],
                      read_origin=st.origins[i]) for i in range(n_read)]
        b = ctx.upload(pairs)
        flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
        b.run(cfg, prm.resolution, flags)
        nb = dict(launches=0, total_ms=0.0, bytes=0.0)
        reps = max(3, args.steps)
        tb = time.perf_counter()
        for _ in range(reps):
            b.run(cfg, prm.resolution, flags | L.AICP_RUN_TIME_NN)
            t = ctx.last_nn_timing()
            for k in ("launches", "total_ms", "bytes"):
                nb[k] += t[k]
        dtb = time.perf_counter() - tb
        b.free()
        batched = {"clouds_per_s": round(reps * n_read / dtb, 3), "ms_per_step": round(1e3 * dtb / reps, 3),
                   "roofline_nn": roofline_nn(nb, "k_icp_nn"),
                   "note": "the same 64 readings as independent pairs against uncorrected references, all "
                           "windows at once, inputs resident in HBM (aicp_hip_batch_run); not the stream's "
                           "dependency chain, so not the headline"}
    if rank == 0:
        value = world * n_read * args.steps / elapsed
        config = {"workload": "%s: App frame-to-reference stream, %s batch_size=80 clouds, N=M=%d, first cloud + "
                              "%d readings, reference = every %dth accepted reading corrected on the device, "
                              "max_correction_magnitude %.1f" % (
                                  args.config.upper(), "ANYmal VLP-16" if args.config == "c2" else "KITTI HDL-64",
                                  n_pts, n_read, args.ref_every, prm.max_correction_magnitude),
                  "readings_per_step_per_gpu": n_read, "windows_per_step": windows, "replans": replans,
                  "working_mode": args.working_mode,
                  "raw_clouds": bool(args.raw),
                  "chain": CHAIN, "overlap": "octree-equivalent voxel sets at 0.2 m",
                  "timed_region": ("raw host clouds -> device pre-filter (App's order) -> stream -> corrections "
                                   "(aicp_hip_sequence_run_raw)" if args.raw else
                                   "host clouds -> packing -> H2D -> device -> corrections (aicp_hip_sequence_run)"),
                  "parallelism": "one stream per rank (replicas), RCCL all_gather of T"}
        out_line = base_line(args, world, METRIC, value, "aligned clouds/s", 1e3 * elapsed / args.steps, DTYPE, DATA,
                             config)
        if args.data:
            config["workload"] = "recorded stream %s: first cloud + %d readings (mean N=%d), reference every %d" % (
                os.path.basename(os.path.abspath(args.data)), n_read, n_pts, args.ref_every)
            out_line["data"] = "recorded (%s)" % args.data
        errs = [sy.rot_err(Tg, Tx) for Tg, Tx in zip(st.T_gt, T) if Tg is not None] or [(float("nan"),) * 2]
        out_line.update({
            "icp_iters_per_s": round(iters / elapsed, 1),
            "mean_iterations": float(np.mean([o["icp"]["iterations"] for o in out])),
            "device_ms_per_step": round(dev_ms / args.steps, 3),
            "call_wall_ms_per_step": round(wall_ms / args.steps, 3),
            "accuracy_vs_ground_truth": {"median_rot_rad": float(np.median([e[0] for e in errs])),
                                         "median_trans_m": float(np.median([e[1] for e in errs])),
                                         "note": "the reference chain (eps 3.16 approximate NN) stalls on this "
                                                 "scene; the oracle gives the same transforms (parity_vs_oracle), "
                                                 "and with eps 0 the oracle reaches the ground truth "
                                                 "(tests/test_oracle.py::test_c2_stall_is_the_epsilon_approximation"
                                                 ", DESIGN.md §7)"},
            "roofline": roofline_nn(nn, "k_icp_nn (transform + libnabo-order 1-NN over treelets + bucket scan), "
                                        "one launch per ICP iteration of a reference window (5 readings)"),
            "batched_independent": batched,
        })
        add_traffic(out_line["roofline"], "nn_traffic_%s.json" % args.config)
        if world == 1 and not args.no_cpu_baseline:
            out_line["cpu_baseline"], out_line["parity_vs_oracle"] = cpu_stream(st, T, out, args)
        print(json.dumps(out_line))
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_stream(st, T, out, args):
    """The oracle's replay of App::processCloud on the first 6 readings of the same stream (one
    reference window + the first reading registered against a corrected reading), 5 times:
    median rate, and parity of those readings' corrections with the device's."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    from aicp_mapping_amd import synthetic as sy

    po.lib()
    k = min(6, len(st.readings))
    res = float(np.float32(0.2))
    last = {}

    def rep():
        t = time.perf_counter()
        last["r"] = po.sequence(st.first, st.first_origin, st.readings[:k], st.origins[:k],
                                reference_update_frequency=args.ref_every, resolution=res,
                                working_mode=args.working_mode, prefilter_with=True if args.raw else None)
        return k, time.perf_counter() - t

    med, rates = median_rate(rep, args.cpu_reps)
    pe = [sy.rot_err(r["T"], T[i]) for i, r in enumerate(last["r"])]
    same = all(r["is_reference"] == out[i]["is_reference"] and r["accepted"] == out[i]["accepted"] and
               r["stats"].iterations == out[i]["icp"]["iterations"] for i, r in enumerate(last["r"]))
    cb = {"value": med, "unit": "aligned_clouds/s", "cores": 1, "kind": "port",
          "sample": "oracle replay of App's stream on readings 0..%d of the same workload (%soverlap + ratio + ICP, "
                    "reference update after reading %d), N=%d, on 1 host core (%s, nproc %d); median of %d runs: %s "
                    "clouds/s" % (k - 1, "pre-filter + " if args.raw else "", args.ref_every - 1, len(st.readings[0]), cpu_model(), os.cpu_count(),
                                  len(rates), ", ".join("%.3f" % r for r in rates))}
    par = {"readings": k, "max_rot_rad": max(e[0] for e in pe), "max_trans_m": max(e[1] for e in pe),
           "same_decisions_and_iterations": bool(same), "tol": [1e-4, 1e-3]}
    return cb, par


def bench_c4(args):
    """C4: localization against a resident 1 M-point map; per step the 64 host readings go in, the
    device crops each reference out of the map (aicp_hip_map_register_batch), T comes out."""
    import aicp_mapping_amd._lib as L
    from aicp_mapping_amd import sharding as sh
    from aicp_mapping_amd import synthetic as sy
    from aicp_mapping_amd.prior_map import PriorMap

    rank, world, local_rank, dist = init_dist()
    n_read = args.pairs or 64
    n_pts = args.points or 120000
    mp, reads, poses, gts = make_c4(n_read, n_pts, 1000000, seed=1 + rank)
    ctx = L.Context(local_rank)
    pm = PriorMap(ctx, mp)  # the prior map is loaded once (App: loadMapFromFile)
    cfg = L.default_config()

    def step():
        return pm.register_batch(reads, poses, -15.0, 15.0, cfg, flags=L.AICP_RUN_TIME_NN)

    for _ in range(args.warmup):
        step()
    sync(dist)
    nn = dict(launches=0, total_ms=0.0, bytes=0.0)
    iters = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        T, st, rc = step()
        t = ctx.last_nn_timing()
        for k in ("launches", "total_ms", "bytes"):
            nn[k] += t[k]
        iters += sum(s["iterations"] for s in st)
    sync(dist)
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = sh.max_over_ranks(elapsed, dist, device="cuda")
    if rank == 0:
        value = world * n_read * args.steps / elapsed
        crops = [len(pm.crop(-15.0, 15.0, poses[i])) for i in (0, n_read - 1)]
        config = {"workload": "C4: localization-only, %d-pt map resident on the device, %d VLP-16 readings of N=%d, "
                              "reference = map cropped to +-15 m around each prior pose on the device "
                              "(getPointsInOrientedBox), overlap fixed 50%% (r = 0.5)" % (len(mp), n_read, n_pts),
                  "map_points": len(mp), "crop_points_first_last": crops, "chain": CHAIN,
                  "timed_region": "host readings -> H2D -> device crops + registration -> T "
                                  "(aicp_hip_map_register_batch)",
                  "parallelism": "one stream per rank (replicas)"}
        line = base_line(args, world, METRIC, value, "aligned clouds/s", 1e3 * elapsed / args.steps, DTYPE, DATA,
                         config)
        errs = [sy.rot_err(g, Tx) for g, Tx in zip(gts, T)]
        line.update({"icp_iters_per_s": round(iters / elapsed, 1),
                     "mean_iterations": float(np.mean([s["iterations"] for s in st])),
                     "accuracy_vs_ground_truth": {"median_rot_rad": float(np.median([e[0] for e in errs])),
                                                  "median_trans_m": float(np.median([e[1] for e in errs]))},
                     "roofline": roofline_nn(nn, "k_icp_nn, one launch per ICP iteration of the 64-reading batch")})
        if world == 1 and not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import pyoracle as po

            po.lib()
            k = 2
            last = {}

            def rep():
                t = time.perf_counter()
                last["T"] = []
                for i in range(k):
                    crop, _ = po.crop_box(mp, -15.0, 15.0, poses[i])
                    last["T"].append(po.icp(crop, reads[i], po.default_config(trimmed_ratio=0.5))[1])
                return k, time.perf_counter() - t

            med, rates = median_rate(rep, args.cpu_reps)
            pe = [sy.rot_err(To, T[i]) for i, To in enumerate(last["T"])]
            line["cpu_baseline"] = {"value": med, "unit": "aligned_clouds/s", "cores": 1, "kind": "port",
                                    "sample": "oracle crop + ICP of readings 0..%d of the same workload on 1 host core "
                                              "(%s, nproc %d); median of %d runs: %s" % (
                                                  k - 1, cpu_model(), os.cpu_count(), len(rates),
                                                  ", ".join("%.3f" % r for r in rates))}
            line["parity_vs_oracle"] = {"pairs": k, "max_rot_rad": max(e[0] for e in pe),
                                        "max_trans_m": max(e[1] for e in pe), "tol": [1e-4, 1e-3]}
        print(json.dumps(line))
    pm.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def bench_c5(args):
    """C5: 1024 independent pairs sharded i mod G; per step a rank's pairs go in from host buffers
    and the transforms come out (aicp_hip_align_batch), RCCL all-gathers the records."""
    import aicp_mapping_amd._lib as L
    from aicp_mapping_amd import sharding as sh
    from aicp_mapping_amd import synthetic as sy

    rank, world, local_rank, dist = init_dist()
    n_total = args.pairs or 1024
    n_pts = args.points or 60000
    pairs = make_c5_pairs(n_total, n_pts, rank, world)
    mine = sh.shard_pairs(n_total, world, rank)
    ctx = L.Context(local_rank)
    cfg = L.default_config()
    res = float(np.float32(0.2))
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP

    def step():
        T, st, rc = ctx.align_batch(pairs, cfg, res, flags | L.AICP_RUN_TIME_NN)
        if dist is not None:
            rec = sh.pack_records(T.transpose(0, 2, 1).reshape(-1, 16), [s["iterations"] for s in st],
                                  [s["inlier_ratio"] for s in st])
            sh.gather_records(rec, dist, device="cuda", pair_index=mine)
        return T, st

    for _ in range(args.warmup):
        step()
    sync(dist)
    nn = dict(launches=0, total_ms=0.0, bytes=0.0)
    iters = 0
    t0 = time.perf_counter()
    for _ in range(args.steps):
        T, st = step()
        t = ctx.last_nn_timing()
        for k in ("launches", "total_ms", "bytes"):
            nn[k] += t[k]
        iters += sum(s["iterations"] for s in st)
    sync(dist)
    elapsed = time.perf_counter() - t0
    # the same batch with its inputs resident in HBM (aicp_hip_batch_upload once, then
    # aicp_hip_batch_run per step): the device-only rate beside the host-buffer `value`
    b = ctx.upload([{k: v for k, v in p.items() if k != "T_gt"} for p in pairs])
    b.run(cfg, res, flags)
    sync(dist)
    t1 = time.perf_counter()
    for _ in range(args.steps):
        b.run(cfg, res, flags)
    sync(dist)
    resident = time.perf_counter() - t1
    same = bool(np.array_equal(b.transforms(), T))
    b.free()
    if dist is not None:
        elapsed = sh.max_over_ranks(elapsed, dist, device="cuda")
        resident = sh.max_over_ranks(resident, dist, device="cuda")
        iters = int(sh.sum_over_ranks(float(iters), dist, device="cuda"))
    if rank == 0:
        value = n_total * args.steps / elapsed
        config = {"workload": "C5: %d independent KITTI-like pairs, N=M=%d, seeds 1000.., sharded i mod G" % (
                  n_total, n_pts), "pairs_total": n_total, "pairs_per_gpu": len(pairs), "chain": CHAIN,
                  "timed_region": "host pairs -> H2D -> overlap + ratio + ICP -> T (aicp_hip_align_batch)",
                  "parallelism": "pairs sharded i mod G, RCCL all_gather of T"}
        line = base_line(args, world, METRIC, value, "aligned clouds/s", 1e3 * elapsed / args.steps, DTYPE, DATA,
                         config, scaling="strong")
        errs = [sy.rot_err(p["T_gt"], Tx) for p, Tx in zip(pairs, T)]
        line.update({"icp_iters_per_s": round(iters / elapsed, 1),
                     "mean_iterations": float(np.mean([s["iterations"] for s in st])),
                     "accuracy_vs_ground_truth": {"median_rot_rad": float(np.median([e[0] for e in errs])),
                                                  "median_trans_m": float(np.median([e[1] for e in errs]))},
                     "roofline": roofline_nn(nn, "k_icp_nn, one launch per ICP iteration of the 1024-pair batch"),
                     "inputs_resident": {"clouds_per_s": round(n_total * args.steps / resident, 1),
                                         "ms_per_step": round(1e3 * resident / args.steps, 3),
                                         "same_transforms": same,
                                         "note": "aicp_hip_batch_upload once, aicp_hip_batch_run per step: "
                                                 "no packing or H2D in the timed region"}})
        add_traffic(line["roofline"], "nn_traffic_c5.json")
        if world == 1 and not args.no_cpu_baseline:
            line["cpu_baseline"], line["cpu_baseline_all_cores"], line["parity_vs_oracle"] = cpu_c5(pairs, T, args)
        print(json.dumps(line))
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


def cpu_c5(pairs, T, args):
    """The oracle on C5 pairs: 1 core (median of 5 samples of 4 pairs) and all of this rank's
    host-core share (16 threads, one pair per thread at a time, ctypes releases the GIL; median of
    5 samples of 64 pairs)."""
    from concurrent.futures import ThreadPoolExecutor

    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po
    from aicp_mapping_amd import synthetic as sy

    po.lib()
    res = float(np.float32(0.2))

    def one(p):
        ov, _ = po.overlap(p["ref"], p["ref_origin"], p["read"], p["read_origin"], res)
        return po.icp(p["ref"], p["read"], po.default_config(trimmed_ratio=po.autotune_ratio(ov)))[1]

    last = {}

    def rep1():
        t = time.perf_counter()
        last["T"] = [one(p) for p in pairs[:4]]
        return 4, time.perf_counter() - t

    med1, r1 = median_rate(rep1, args.cpu_reps)
    threads = min(16, os.cpu_count() or 1)
    sub = pairs[:64]

    def repn():
        t = time.perf_counter()
        with ThreadPoolExecutor(max_workers=threads) as ex:
            list(ex.map(one, sub))
        return len(sub), time.perf_counter() - t

    medn, rn = median_rate(repn, args.cpu_reps)
    pe = [sy.rot_err(To, T[i]) for i, To in enumerate(last["T"])]
    cb1 = {"value": med1, "unit": "aligned_clouds/s", "cores": 1, "kind": "port",
           "sample": "oracle overlap + ratio + ICP of the first 4 pairs on 1 host core (%s, nproc %d); median of %d "
                     "runs: %s" % (cpu_model(), os.cpu_count(), len(r1), ", ".join("%.3f" % r for r in r1))}
    cbn = {"value": medn, "unit": "aligned_clouds/s", "cores": threads, "kind": "port",
           "sample": "the same on the first 64 pairs, one pair per thread on %d threads (the box's host-core share "
                     "per GPU; nproc %d); median of %d runs: %s" % (threads, os.cpu_count(), len(rn),
                                                                   ", ".join("%.3f" % r for r in rn))}
    par = {"pairs": len(pe), "max_rot_rad": max(e[0] for e in pe), "max_trans_m": max(e[1] for e in pe),
           "tol": [1e-4, 1e-3]}
    return cb1, cbn, par


def bench_single(args):
    """The call App actually makes: one pair per registerClouds (app.cpp:210, 528-550), host
    buffers -> T through aicp_hip_register; latency median over the timed steps, next to the
    oracle's on the same pair."""
    import aicp_mapping_amd._lib as L
    from aicp_mapping_amd import synthetic as sy

    n_pts = args.points or 120000
    first, o0 = sy.stream_first(1, n_pts)
    read, origin, Tg = sy.stream_reading(1, 0, n_pts)
    ctx = L.Context(0)
    cfg = L.default_config()
    # `value`: every call with a reference and a reading the context has not seen last (two copies
    # of each, alternated: a new pointer is a new cloud, so nothing is served from the resident
    # reference of DESIGN 5.2); the same pair called again (App's readings 2-5 of a window reuse
    # the reference, not the reading) is reported beside it as latency_ms_resident
    refs, reads = [first, first.copy()], [read, read.copy()]
    for i in range(max(1, args.warmup)):
        ctx.register(refs[i % 2], reads[i % 2], cfg)
    lat = []
    for i in range(max(5, args.steps)):
        t = time.perf_counter()
        T1, s1 = ctx.register(refs[i % 2], reads[i % 2], cfg)  # aicp_hip_register: host xyz -> T
        lat.append(time.perf_counter() - t)
    warm = []
    for _ in range(max(5, args.steps)):
        t = time.perf_counter()
        Tw, _ = ctx.register(first, reads[0], cfg)
        warm.append(time.perf_counter() - t)
    assert np.array_equal(Tw, T1), "a resident reference changed the result"
    T, st = T1[None], [s1]
    med = float(np.median(lat))
    line = base_line(args, 1, "single-pair registration latency (aicp_hip_register, host xyz -> T)", 1e3 * med, "ms",
                     1e3 * med, DTYPE, DATA,
                     {"workload": "one C2 pair (first cloud vs reading 0 of the C2 stream), N=M=%d, ratio 0.70 "
                                  "(registerClouds re-reads the chain; no overlap in this call)" % n_pts,
                      "chain": CHAIN}, scaling="strong", hib=False)
    line.update({"latency_ms_samples": [round(1e3 * x, 3) for x in lat], "iterations": st[0]["iterations"],
                 "latency_ms_resident": {"median": round(1e3 * float(np.median(warm)), 3),
                                         "note": "the same pair again: reference and reading resident "
                                                 "(aicp_hip_reference_cache_stats hits)"}})
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as po

        po.lib()
        lo = []
        for _ in range(args.cpu_reps):
            t = time.perf_counter()
            rc1, To, sto = po.icp(first, read, po.default_config(trimmed_ratio=0.7))
            lo.append(time.perf_counter() - t)
        r, tt = sy.rot_err(To, T[0])
        line["cpu_baseline"] = {"value": 1e3 * float(np.median(lo)), "unit": "ms", "cores": 1, "kind": "port",
                                "sample": "the oracle's ICP of the same pair on 1 host core (%s), median of %d: %s ms"
                                          % (cpu_model(), len(lo), ", ".join("%.1f" % (1e3 * x) for x in lo))}
        line["parity_vs_oracle"] = {"rot_rad": r, "trans_m": tt, "iterations_equal": sto.iterations ==
                                    st[0]["iterations"], "tol": [1e-4, 1e-3]}
    print(json.dumps(line))
    ctx.close()


def bench_app(args):
    """The drop-in path as App drives it (app.cpp:282-414 robot mode, through the shim of
    INTEGRATION.md): per reading computeOverlap (aicp_hip_overlap), the auto-tuned ratio
    (app.cpp:197-205), registerClouds (aicp_hip_register), the max-correction drop
    (app.cpp:366-373), and every 5th accepted reading, corrected by getOutputReading
    (aicp_hip_transform), becomes the reference with its corrected pose as origin
    (app.cpp:375-391). Host xyz in, T out, one call at a time: the reference side stays resident
    between the calls of a window (aicp_hip_reference_cache_stats). Reports the per-reading latency
    of window readings 2..5 (reference reused) and of the window's first reading (reference
    built), and aligned clouds/s over the whole stream."""
    import aicp_mapping_amd._lib as L
    from aicp_mapping_amd import registration as R
    from aicp_mapping_amd import synthetic as sy

    n_read = args.pairs or 64
    n_pts = args.points or 120000
    st = make_stream(n_read, n_pts, seed=1)
    ctx = L.Context(0)
    res = float(np.float32(0.2))
    max_corr = 1.0

    split = []  # reused-reference readings: overlap call, register call, the register's phases

    def run():
        ref, ref_o = st.first, np.asarray(st.first_origin, np.float64)
        acc = 0
        lat, first_lat, Ts, its = [], [], [], []
        for i, (r, o) in enumerate(zip(st.readings, st.origins)):
            t = time.perf_counter()
            ov = ctx.overlap(ref, r, ref_o, o, res)
            t1 = time.perf_counter()
            cfg = L.default_config(trimmed_ratio=L.autotune_ratio(ov))
            T, s1 = ctx.register(ref, r, cfg)
            t2 = time.perf_counter()
            dt = t2 - t
            (first_lat if acc == 0 else lat).append(dt)
            if acc:
                split.append((t1 - t, t2 - t1, ctx.last_phase_ms()))
            Ts.append(T)
            its.append(s1["iterations"])
            if np.linalg.norm(T[:3, 3]) > max_corr:  # dropped (app.cpp:366-373)
                continue
            acc += 1
            if acc == args.ref_every:  # the corrected reading becomes the reference (app.cpp:375-391)
                ref = ctx.transform(T, r)
                ref_o = (R.isometry_from_matrix4f(T) @ np.r_[np.asarray(o, np.float64), 1.0])[:3]
                acc = 0
        return lat, first_lat, Ts, its

    for _ in range(args.warmup):
        run()
    c0 = ctx.reference_cache_stats()
    t0 = time.perf_counter()
    lat, first_lat = [], []
    for _ in range(args.steps):
        l, f, Ts, its = run()
        lat += l
        first_lat += f
    elapsed = time.perf_counter() - t0
    c1 = ctx.reference_cache_stats()
    value = n_read * args.steps / elapsed
    line = base_line(args, 1, METRIC + " -- drop-in call path (overlap + registerClouds per reading)", value,
                     "aligned clouds/s", 1e3 * elapsed / args.steps, DTYPE, DATA,
                     {"workload": "C2 readings through App's per-reading calls (aicp_hip_overlap + aicp_hip_register, "
                                  "reference = every %dth accepted reading corrected by aicp_hip_transform), N=M=%d, "
                                  "%d readings" % (args.ref_every, n_pts, n_read),
                      "chain": CHAIN, "timed_region": "host xyz -> overlap -> ratio -> registerClouds -> T, per call"},
                     scaling="strong")
    line.update({
        "reading_ms_reference_reused": {"median": round(1e3 * float(np.median(lat)), 3),
                                        "p90": round(1e3 * float(np.percentile(lat, 90)), 3), "n": len(lat)},
        "reading_ms_reference_built": {"median": round(1e3 * float(np.median(first_lat)), 3), "n": len(first_lat)},
        "reference_cache": {k: int(c1[k] - c0[k]) for k in c1},
        "reused_split_ms": {"overlap_call": round(1e3 * float(np.median([x[0] for x in split])), 3),
                            "register_call": round(1e3 * float(np.median([x[1] for x in split])), 3),
                            "register_icp_loop_device": round(float(np.median([x[2]["icp_loop"] for x in split])), 3)},
        "mean_iterations": float(np.mean(its)),
    })
    if not args.no_cpu_baseline:
        sys.path.insert(0, os.path.join(ROOT, "oracle"))
        import pyoracle as po

        po.lib()
        k = min(6, n_read)
        ref = po.sequence(st.first, st.first_origin, st.readings[:k], st.origins[:k], reference_update_frequency=
                          args.ref_every, resolution=res)
        pe = [sy.rot_err(x["T"], Ts[i]) for i, x in enumerate(ref)]
        line["parity_vs_oracle"] = {"readings": k, "max_rot_rad": max(e[0] for e in pe),
                                    "max_trans_m": max(e[1] for e in pe),
                                    "iterations_equal": all(x["stats"].iterations == its[i] for i, x in enumerate(ref)),
                                    "tol": [1e-6, 1e-5]}
    print(json.dumps(line))
    ctx.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5", "single", "app", "prefilter"], default="c2",
                    help="BASELINE.json workload (default c2: the metric's configuration)")
    ap.add_argument("--pairs", type=int, default=None, help="readings (pairs) per step per GPU")
    ap.add_argument("--ref-every", type=int, default=5, help="reference_update_frequency")
    ap.add_argument("--working-mode", choices=["robot", "debug"], default="robot",
                    help="App's working_mode for c2/c3 (debug: readings pre-transformed by initialT_, serial)")
    ap.add_argument("--raw", action="store_true",
                    help="c2/c3: the clouds are raw; App's pre-filter runs in App's order inside the timed "
                         "region (aicp_hip_sequence_run_raw)")
    ap.add_argument("--points", type=int, default=None)
    ap.add_argument("--data", default=None,
                    help="recorded directory (aicp_input_poses.csv + cloud_*.pcd) replayed as the stream")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--cpu-reps", type=int, default=5, help="repetitions of the bounded CPU sample (median)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-batched", action="store_true", help="skip the batched-independent extra figure")
    ap.add_argument("--opt", action="append", default=[], metavar="K=V",
                    help="context option (aicp_hip_options, include/aicp_hip.h) for every context, e.g. profile=1")
    args = ap.parse_args()
    if args.opt:
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        import aicp_mapping_amd._lib as L

        for kv in args.opt:
            k, _, v = kv.partition("=")
            L.CONTEXT_OPTIONS[k.strip()] = int(v)
    if args.config == "prefilter":
        return bench_prefilter(args)
    if args.config in ("c2", "c3"):
        return bench_stream(args)
    if args.config == "c4":
        return bench_c4(args)
    if args.config == "c5":
        return bench_c5(args)
    if args.config == "app":
        return bench_app(args)
    return bench_single(args)


if __name__ == "__main__":
    main()
