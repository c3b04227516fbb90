#!/usr/bin/env python3
"""Benchmark: aligned clouds/s (+ ICP iterations/s) on the C2 workload.

C2 = ANYmal VLP-16 clouds of the batch_size = 80 accumulation (aicp_ros_node.cpp:40),
N = M = 120 000 points, registered frame-to-reference in a streamed sequence of 64 readings
with the reference replaced every 5 readings (aicp.launch reference_update_frequency). A step
= one such sequence run end to end on the GPU: per pair octree overlap -> auto-tuned trimmed
ratio -> ICP; per reference window centroid + kd-tree + SurfaceNormal built once (§8(f)
rank 1). Inputs are resident in HBM before timing (aicp_hip_batch_upload); each rank
registers its own sequence (weak scaling) and RCCL all-gathers the per-pair {T, iterations,
inlier ratio}.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--pairs 64] [--ref-every 5] [--points N]
    torchrun --nproc-per-node N bench.py --gpus N ...
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


def make_pairs(n_readings, ref_every, n_points, seed):
    from aicp_mapping_amd import synthetic as sy

    return [dict(ref=pr.ref, read=pr.read, ref_origin=pr.ref_origin, read_origin=pr.read_origin, T_gt=pr.T_gt)
            for pr in sy.make_sequence(n_readings, ref_every, n_points, seed=seed)]


def _c5_pair(seed_points):
    from aicp_mapping_amd import synthetic as sy

    seed, n = seed_points
    pr = sy.make_pair(n, n, seed=seed)
    return dict(ref=pr.ref, read=pr.read, ref_origin=pr.ref_origin, read_origin=pr.read_origin, T_gt=pr.T_gt)


def make_c5_pairs(n_total, n_points, rank, world):
    """C5: independent pairs, seeds 1000..; rank g takes pairs i = g mod G
    (sharding.shard_pairs). Generated in a process pool (16 workers: the box's CPU share)."""
    from concurrent.futures import ProcessPoolExecutor

    from aicp_mapping_amd import sharding as sh

    mine = sh.shard_pairs(n_total, world, rank)
    with ProcessPoolExecutor(max_workers=min(16, os.cpu_count() or 1)) as ex:
        return list(ex.map(_c5_pair, [(1000 + i, n_points) for i in mine], chunksize=4))


def make_c4_pairs(n_readings, n_points, map_points, crop, seed):
    """C4 localization-only: a resident map of map_points points over the whole
    scene; reading i (N points, sensor moving along x) registers against the map points within
    +-crop m of its prior position (the cropped map, M ~ 250k); overlap fixed at 50 % => r = 0.5.
    The crop is input preparation here (an axis-aligned box around the prior position)."""
    from aicp_mapping_amd import synthetic as sy

    seq = sy.make_sequence(n_readings, n_readings, n_points, seed=seed)
    scene = sy.make_scene(seed)
    rng = np.random.default_rng(seed * 7919 + 77)
    mp = sy.sample_scene(scene, rng, np.array([0.0, 0.0, 0.7]), half=40.0)
    if len(mp) > map_points:
        mp = mp[rng.choice(len(mp), size=map_points, replace=False)]
    mp = mp.astype(np.float32)
    out = []
    for i, pr in enumerate(seq):
        o = np.array([(i + 1) * 0.3, 0.0, 0.7])  # prior position of reading i (make_sequence's path)
        m = np.all(np.abs(mp - o.astype(np.float32)) <= crop, axis=1)
        ref = np.ascontiguousarray(mp[m])
        out.append(dict(ref=ref, read=pr.read, ref_origin=o, read_origin=pr.read_origin, T_gt=pr.T_gt))
    return out, len(mp)


def cpu_baseline(pairs, res, budget_s, cfg_ratio, run_overlap, workload):
    """The oracle (single-thread C++ restatement of the libpointmatcher chain) on a bounded sample
    of the same workload as the GPU run: whole pairs, as many as fit the budget. With the overlap
    (C2, C3, C5) each pair runs overlap -> auto-tuned ratio -> ICP like the device; without it
    (C4: localization against the map, overlap fixed) ICP runs at the configured ratio."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import pyoracle as po

    po.lib()
    done = 0
    iters = 0
    Ts = []
    t0 = time.perf_counter()
    for p in pairs:
        ratio = cfg_ratio
        if run_overlap:
            ov, _ = po.overlap(p["ref"], p["ref_origin"], p["read"], p["read_origin"], res)
            ratio = po.autotune_ratio(ov)
        rc, T, st = po.icp(p["ref"], p["read"], po.default_config(trimmed_ratio=ratio))
        Ts.append(T)
        done += 1
        iters += st.iterations
        if time.perf_counter() - t0 > budget_s:
            break
    dt = time.perf_counter() - t0
    steps = "overlap + ratio + ICP" if run_overlap else "ICP at r = %.2f" % cfg_ratio
    return dict(value=done / dt, unit="aligned_clouds/s", cores=1, kind="port",
                sample=f"first {done} pair(s) of [{workload}] ({steps}, N={pairs[0]['read'].shape[0]}, "
                       f"M={pairs[0]['ref'].shape[0]}) on 1 host core ({cpu_model()}, nproc {os.cpu_count()}); "
                       f"{iters} ICP iterations in {dt:.1f} s",
                icp_iters_per_s=iters / dt), Ts


def load_traffic():
    path = os.path.join(ROOT, "profiles", "nn_traffic.json")
    if os.path.exists(path):
        try:
            return json.load(open(path))
        except (OSError, ValueError):
            return None
    return None


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


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", choices=["c2", "c3", "c4", "c5", "prefilter"], default="c2",
                    help="BASELINE.json workload (default c2: the metric's configuration); prefilter: the "
                         "SURVEY §8(f) rank 2 pre-filter on C2's raw clouds")
    ap.add_argument("--pairs", type=int, default=None, help="readings (pairs) per step per GPU")
    ap.add_argument("--ref-every", type=int, default=5, help="readings per reference window")
    ap.add_argument("--data", default=None,
                    help="recorded directory (aicp_input_poses.csv + cloud_*.pcd) replayed instead of "
                         "synthetic C2 clouds; the workload then names the directory")
    ap.add_argument("--points", type=int, default=None)
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--lanes", type=int, default=1,
                    help="independent copies of the step in flight on the GPU (each its own context, streams "
                         "and resident batch, driven by its own host thread); the K timed steps are shared out")
    args = ap.parse_args()
    if args.config == "prefilter":
        return bench_prefilter(args)

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

    res = float(np.float32(0.2))  # octomapResolution read as<float> (yaml_configurator.cpp:81)
    cfg = L.default_config()
    flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
    extra = {}
    if args.data:
        from aicp_mapping_amd import cloud_io

        pairs = cloud_io.recorded_sequence_pairs(args.data, args.ref_every, args.pairs)
        if not pairs:
            raise SystemExit(f"--data {args.data}: no readable pose/cloud pairs")
        args.pairs = len(pairs)
        args.points = int(np.mean([len(p["read"]) for p in pairs]))
        workload = "recorded sequence %s: %d readings (mean N=%d), reference updated every %d" % (
            os.path.basename(os.path.abspath(args.data)), args.pairs, args.points, args.ref_every)
    elif args.config in ("c2", "c3"):
        args.pairs = args.pairs or 64
        args.points = args.points or (120000 if args.config == "c2" else 600000)
        # each rank streams its own sequence (seed 1 + rank): weak scaling over independent pairs
        pairs = make_pairs(args.pairs, args.ref_every, args.points, seed=1 + rank)
        workload = ("%s: %s batch_size=80 clouds, N=M=%d, frame-to-reference sequence of %d readings, "
                    "reference updated every %d" % (args.config.upper(), "ANYmal VLP-16" if args.config == "c2"
                                                    else "KITTI HDL-64", args.points, args.pairs, args.ref_every))
    elif args.config == "c4":
        args.pairs = args.pairs or 64
        args.points = args.points or 120000
        pairs, n_map = make_c4_pairs(args.pairs, args.points, 1000000, 15.0, seed=1 + rank)
        cfg = L.default_config(trimmed_ratio=0.5)  # overlap fixed at 50 % (app.cpp:123-127)
        flags = L.AICP_RUN_ICP
        extra = {"map_points": n_map, "mean_ref_points": int(np.mean([len(p["ref"]) for p in pairs]))}
        workload = ("C4: localization-only, %d-pt map cropped to +-15 m per reading, %d VLP-16 readings of "
                    "N=%d, r=0.5" % (n_map, args.pairs, args.points))
    else:
        args.points = args.points or 60000
        n_total = args.pairs or 1024
        pairs = make_c5_pairs(n_total, args.points, rank, world)
        args.pairs = len(pairs)
        extra = {"pairs_total": n_total}
        workload = "C5: %d independent KITTI-like pairs, N=M=%d, seeds 1000.., sharded i mod G" % (
            n_total, args.points)
    order = os.environ.get("AICP_BENCH_READ_ORDER")  # experiment: host-side reading order
    if order:
        rng = np.random.default_rng(0)
        for p in pairs:
            r = p["read"]
            if order == "shuffle":
                idx = rng.permutation(len(r))
            else:  # morton on 0.25 m cells
                q = (np.floor(r / 0.25).astype(np.int64) & 1023)
                key = np.zeros(len(r), np.int64)
                for b in range(10):
                    for a in range(3):
                        key |= ((q[:, a] >> b) & 1) << (3 * b + a)
                idx = np.argsort(key, kind="stable")
            p["read"] = np.ascontiguousarray(r[idx])
    n_refs = len({id(p["ref"]) for p in pairs})
    ctx = L.Context(local_rank)
    batch = ctx.upload(pairs)

    # global index of each local pair for the result gather (C5: the i mod G shard; the other
    # configs: every rank its own sequence, rank-major)
    pair_index = (sh.shard_pairs(extra["pairs_total"], world, rank) if args.config == "c5" and not args.data
                  else None)

    def gather():
        if dist is None:
            return None
        st = batch.stats
        rec = sh.pack_records(batch.outT, [s.iterations for s in st], [s.inlier_ratio for s in st])
        return sh.gather_records(rec, dist, device="cuda", pair_index=pair_index)

    def sync():
        if dist is not None:
            import torch

            torch.cuda.synchronize()
            dist.barrier()

    for _ in range(args.warmup):
        batch.run(cfg, res, flags)
        gather()
    sync()
    nn_ms = nn_bytes = 0.0
    nn_launches = 0
    iters_total = 0
    phases = np.zeros(5)
    lanes = max(1, args.lanes)
    if lanes > 1:
        # further copies of the same step, each on its own context (streams, buffers, resident
        # batch) and host thread, so one copy's tree builds and small ICP kernels fill the chip
        # while another's NN launches run; the K timed steps are shared out lane by lane
        import queue
        import threading

        lane_ctx = [(ctx, batch)]
        for _ in range(lanes - 1):
            c2 = L.Context(local_rank)
            b2 = c2.upload(pairs)
            for _ in range(max(1, args.warmup)):
                b2.run(cfg, res, flags)
            lane_ctx.append((c2, b2))
        sync()
        per_lane = [args.steps // lanes + (1 if i < args.steps % lanes else 0) for i in range(lanes)]
        done_q = [queue.Queue() for _ in range(lanes)]

        def lane_main(i):
            c, b = lane_ctx[i]
            for _ in range(per_lane[i]):
                b.run(cfg, res, flags | L.AICP_RUN_TIME_NN)
                done_q[i].put((c.last_nn_timing(), sum(s.iterations for s in b.stats), c.last_phase_ms(),
                               b.outT.copy(), [s.iterations for s in b.stats], [s.inlier_ratio for s in b.stats]))

        t0 = time.perf_counter()
        th = [threading.Thread(target=lane_main, args=(i,)) for i in range(lanes)]
        for x in th:
            x.start()
        for k in range(max(per_lane)):  # results gathered in a fixed (step, lane) order on every rank
            for i in range(lanes):
                if k >= per_lane[i]:
                    continue
                t, it, ph, outT, its, inl = done_q[i].get()
                if dist is not None:
                    sh.gather_records(sh.pack_records(outT, its, inl), dist, device="cuda", pair_index=pair_index)
                nn_ms += t["total_ms"]
                nn_bytes += t["bytes"]
                nn_launches += t["launches"]
                iters_total += it
                phases += np.array([ph["overlap"], ph["normals"], ph["matcher_tree"], ph["icp_loop"], ph["total"]])
        for x in th:
            x.join()
    else:
        t0 = time.perf_counter()
        for _ in range(args.steps):
            batch.run(cfg, res, flags | L.AICP_RUN_TIME_NN)
            gather()
            t = ctx.last_nn_timing()
            nn_ms += t["total_ms"]
            nn_bytes += t["bytes"]
            nn_launches += t["launches"]
            iters_total += sum(s.iterations for s in batch.stats)
            ph = ctx.last_phase_ms()
            phases += np.array([ph["overlap"], ph["normals"], ph["matcher_tree"], ph["icp_loop"], ph["total"]])
    sync()
    elapsed = time.perf_counter() - t0
    if dist is not None:
        elapsed = sh.max_over_ranks(elapsed, dist, device="cuda")
        iters_total = int(sh.sum_over_ranks(float(iters_total), dist, device="cuda"))

    # PCIe-inclusive rate (not `value`): the same step from host buffers, upload + run + free
    # (aicp_hip_align_batch); rank 0 alone, after the timed loop
    pcie = None
    if rank == 0 and not args.data:
        tp = time.perf_counter()
        reps = max(1, min(3, args.steps))
        for _ in range(reps):
            ctx.align_batch(pairs, cfg, res, flags)
        pcie = {"clouds_per_s": round(reps * args.pairs / (time.perf_counter() - tp), 3),
                "note": "host xyz in -> T out per step: H2D of all clouds, run, D2H (aicp_hip_align_batch)"}

    # accuracy of the last step (synthetic ground truth)
    from aicp_mapping_amd import synthetic as sy

    errs = [sy.rot_err(p["T_gt"], T) for p, T in zip(pairs, batch.transforms()) if p["T_gt"] is not None]
    st = batch.stats_dicts()

    if rank == 0:
        total_pairs = (extra.get("pairs_total") or args.pairs * world) * args.steps
        value = total_pairs / elapsed
        avg_launch_ms = nn_ms / max(1, nn_launches)
        achieved = (nn_bytes / max(1, nn_launches)) / (avg_launch_ms * 1e-3) / 1e9 if nn_launches else 0.0
        # the committed PMC figure is per launch of the default C2 workload only
        traffic = load_traffic() if (args.config == "c2" and not args.data) else None
        out = {
            "metric": "aligned_clouds_per_s (ICP iterations/sec + aligned clouds/sec, 80-scan VLP-16 batch)",
            "value": round(value, 3),
            "unit": "aligned clouds/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True,
            "scaling": "strong" if args.config == "c5" else "weak",
            "vs_baseline": None,
            "dtype": "f32 (point arithmetic; 6x6/3x3 reductions and solves in f64)",
            "data": ("recorded (%s)" % args.data) if args.data else
                    "synthetic (seeded planar scene per SURVEY §8(d); no recordings in the reference)",
            "config": {
                "workload": workload,
                "pairs_per_step_per_gpu": args.pairs,
                "references_per_step_per_gpu": n_refs,
                "chain": "icp_autotuned_default.yaml (SurfaceNormal knn20, KDTree knn1 eps3.16, "
                         "TrimmedDist auto-tuned, PointToPlane, Counter20 + Differential)",
                "overlap": "octree-equivalent voxel sets at 0.2 m" if flags & L.AICP_RUN_OVERLAP
                           else "fixed 50 %% (r = %.2f)" % cfg.trimmed_ratio,
                **extra,
                "parallelism": "independent pairs sharded over ranks, RCCL all_gather of T",
                "lanes": lanes,
            },
            "pcie_inclusive": pcie,
            "icp_iters_per_s": round(iters_total / elapsed, 1),
            "mean_iterations": float(np.mean([s["iterations"] for s in st])),
            "phase_ms_per_step": dict(zip(["overlap_gpu (stream 1)", "normal_tree_and_normals_gpu (stream 2)",
                                           "centroid_matcher_tree_gpu (stream 2)", "icp_loop_gpu", "total"],
                                          [round(x / args.steps, 3) for x in phases])),
            "accuracy_vs_ground_truth": {
                "median_rot_rad": float(np.median([e[0] for e in errs])),
                "median_trans_m": float(np.median([e[1] for e in errs])),
                "note": "the reference chain (eps 3.16 approximate NN) stalls in local minima on some "
                        "synthetic pairs; the oracle reproduces the same transforms (parity_vs_oracle)"}
            if errs else None,
            "roofline": {
                "kernel": "k_icp_nn (transform + libnabo-order 1-NN over treelets + bucket scan)",
                "bound": "hbm",
                "achieved": round(achieved, 1),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4),
                "traffic": traffic.get("bytes_per_launch") if traffic else None,
                "avg_launch_us": round(1e3 * avg_launch_ms, 2),
                "algorithmic_bytes_per_launch": round(nn_bytes / max(1, nn_launches)),
                "bytes_model": "N*(12+8) + V*16 + W*8 (SURVEY §8(d)); V, W = touched points / inner nodes",
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            cb, Ts = cpu_baseline(pairs, res, args.cpu_budget, float(cfg.trimmed_ratio),
                                  bool(flags & L.AICP_RUN_OVERLAP), workload)
            out["cpu_baseline"] = cb
            # parity of this run's transforms against the oracle's (reference normal semantics)
            pe = [sy.rot_err(To, Tg) for To, Tg in zip(Ts, batch.transforms())]
            out["parity_vs_oracle"] = {"pairs": len(pe), "max_rot_rad": max(e[0] for e in pe),
                                       "max_trans_m": max(e[1] for e in pe), "tol": [1e-4, 1e-3]}
        print(json.dumps(out))
    batch.free()
    ctx.close()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
