"""Run the device pre-filter on a map-sized synthetic cloud a few times (profiling driver)."""
import sys
import time
import numpy as np
sys.path.insert(0, ".")
from aicp_mapping_amd import synthetic as sy
import aicp_mapping_amd._lib as L
half = float(sys.argv[1]) if len(sys.argv) > 1 else 20.0
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
sc = sy.make_scene(2)
P = sy.sample_scene(sc, np.random.default_rng(102), (0.0, 0.0, 0.7), half=half, spacing=0.035).astype(np.float32)
ctx = L.Context(0)
for r in range(reps):
    t = time.perf_counter()
    d = ctx.prefilter(P, details=False)
    print(f"n {len(P)} out {len(d)} {1e3 * (time.perf_counter() - t):.2f} ms", flush=True)
