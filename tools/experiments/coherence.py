"""Design experiment (not product): how many ICP queries keep their first-descent leaf from one
iteration to the next? For a C2-size pair, the oracle's per-iteration T_iter (matcher frame)
moves every reading point; a query whose displacement is below its descent-path margin (the
smallest |q[cd] - cut| on its root-to-leaf path) provably reaches the same leaf.
Writes /tmp/coh_{ref,read,T}.bin for tools/coherence.cpp."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import pyoracle as po  # noqa: E402
from aicp_mapping_amd import synthetic as sy  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 120000
seed = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
pr = sy.make_pair(n, n, seed=seed)
ov, _ = po.overlap(pr.ref, pr.ref_origin, pr.read, pr.read_origin, float(np.float32(0.2)))
ratio = po.autotune_ratio(ov)
rc, T, st = po.icp(pr.ref, pr.read, po.default_config(trimmed_ratio=ratio, normals_on_centered=0))
it = st.iterations
Ts = np.array([np.array(st.T_iter[k][:]) for k in range(it)], np.float32)
print("iterations", it, "ratio", ratio, "mean", list(st.mean))
pr.ref.astype(np.float32).tofile("/tmp/coh_ref.bin")
pr.read.astype(np.float32).tofile("/tmp/coh_read.bin")
np.concatenate([np.array(st.mean[:], np.float32), Ts.reshape(-1)]).tofile("/tmp/coh_T.bin")
