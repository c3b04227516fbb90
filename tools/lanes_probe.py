"""Probe: the C4 / C5 batch split over L contexts driven from L host threads at once (the library's
calls release the GIL), against one context: clouds/s and whether every transform is identical.
python tools/lanes_probe.py c4|c5 L [steps]"""
import os
import sys
import threading
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402
import aicp_mapping_amd._lib as L  # noqa: E402
from aicp_mapping_amd.prior_map import PriorMap  # noqa: E402

cfgname = sys.argv[1]
lanes = int(sys.argv[2])
steps = int(sys.argv[3]) if len(sys.argv) > 3 else 3
cfg = L.default_config()

if cfgname == "c4":
    mp, reads, poses, gts = bench.make_c4(64, 120000, 1000000, seed=1)
    n = len(reads)

    def make_lane():
        ctx = L.Context(0)
        return ctx, PriorMap(ctx, mp)

    def run(lane, idx):
        ctx, pm = lane
        return pm.register_batch([reads[i] for i in idx], [poses[i] for i in idx], -15.0, 15.0, cfg)[0]
else:
    pairs = [{k: v for k, v in p.items() if k != "T_gt"} for p in bench.make_c5_pairs(1024, 60000, 0, 1)]
    n = len(pairs)

    def make_lane():
        return (L.Context(0),)

    def run(lane, idx):
        return lane[0].align_batch([pairs[i] for i in idx], flags=L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP,
                                   resolution=float(np.float32(0.2)))[0]


def measure(nl):
    ls = [make_lane() for _ in range(nl)]
    parts = [list(range(k, n, nl)) for k in range(nl)]
    out = [None] * nl

    def go():
        th = [threading.Thread(target=lambda k=k: out.__setitem__(k, run(ls[k], parts[k]))) for k in range(nl)]
        for t in th:
            t.start()
        for t in th:
            t.join()

    go()  # warmup
    t0 = time.perf_counter()
    for _ in range(steps):
        go()
    dt = (time.perf_counter() - t0) / steps
    T = np.zeros((n, 4, 4), np.float32)
    for k in range(nl):
        for j, i in enumerate(parts[k]):
            T[i] = out[k][j]
    return n / dt, T


v1, T1 = measure(1)
vl, TL = measure(lanes)
print(cfgname, "1 lane %.1f clouds/s, %d lanes %.1f clouds/s, identical %s" % (v1, lanes, vl, np.array_equal(T1, TL)))
