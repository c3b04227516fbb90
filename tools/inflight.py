"""Experiment: two contexts (own streams and buffers) running C2 batches from two host threads, so
one batch's tree/normal/overlap phase overlaps the other's ICP loop. Prints clouds/s for 1 and 2
in flight."""
import os
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
import aicp_mapping_amd._lib as L  # noqa: E402

pairs = bench.make_pairs(64, 5, 120000, seed=1)
res = float(np.float32(0.2))
cfg = L.default_config()
flags = L.AICP_RUN_OVERLAP | L.AICP_RUN_ICP
n_inflight = int(sys.argv[1]) if len(sys.argv) > 1 else 2
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
ctxs = [L.Context(0) for _ in range(n_inflight)]
batches = [c.upload(pairs) for c in ctxs]
for b in batches:
    b.run(cfg, res, flags)


def worker(b, k):
    for _ in range(k):
        b.run(cfg, res, flags)


t0 = time.perf_counter()
th = [threading.Thread(target=worker, args=(b, steps)) for b in batches]
for t in th:
    t.start()
for t in th:
    t.join()
dt = time.perf_counter() - t0
T0 = batches[0].transforms()
for b in batches[1:]:
    assert np.array_equal(T0, b.transforms())
print(f"in flight {n_inflight}: {n_inflight * steps * 64 / dt:.1f} clouds/s ({dt / steps * 1e3:.2f} ms per round of {n_inflight} batches)")
