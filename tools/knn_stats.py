"""Self-query k-NN traversal statistics on one C2 reference cloud (points and nodes touched per
query, by k), through aicp_hip_knn. Not part of the product.
Usage: python tools/knn_stats.py"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from aicp_mapping_amd import _lib as L  # noqa: E402
from aicp_mapping_amd import synthetic as sy  # noqa: E402

pr = sy.make_sequence(1, 5, 120000, seed=1)[0]
ref = np.ascontiguousarray(pr.ref[:, :3], np.float32)
ctx = L.Context(0)
for k in (1, 4, 10, 20, 30):
    ctx.knn(ref, ref, k=k)
    t0 = time.perf_counter()
    ids, d2, tp, tn = ctx.knn(ref, ref, k=k)
    dt = time.perf_counter() - t0
    n = ref.shape[0]
    print(f"k={k:2d} pts/query {tp / n:7.1f} nodes/query {tn / n:7.1f} call {dt * 1e3:7.2f} ms", flush=True)
ctx.close()
