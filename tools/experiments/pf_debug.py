"""Prefilter GPU vs oracle diagnostics (not part of the product)."""
import sys
import numpy as np
sys.path.insert(0, "."); sys.path.insert(0, "oracle"); sys.path.insert(0, "tests")
from test_prefilter import scene_cloud
import pyoracle as O
import aicp_mapping_amd._lib as L
ctx = L.Context(0)
P = scene_cloud(seed=7, half=5.0)
g = ctx.prefilter(P, details=True)
r = O.prefilter(P)
gs, rs = g["sampled"], r["sampled"]
print("V", len(gs), len(rs), "clusters", g["n_clusters"], r["n_clusters"])
d = np.abs(gs[:, 3:7] - rs[:, 3:7])
print("max abs diff curv/n:", np.nanmax(d, 0))
sign = (np.sign(gs[:, 4:7]) != np.sign(rs[:, 4:7])).any(1)
print("sign flips", sign.sum())
dn = np.abs(np.abs(gs[:, 4:7]) - np.abs(rs[:, 4:7])).max(1)
print("abs-normal diff quantiles", np.quantile(dn, [0.5, 0.9, 0.99, 1.0]))
bad = np.nonzero((gs[:, 3:7] != rs[:, 3:7]).any(1))[0]
print("bad", len(bad))
for i in bad[:4]:
    print(i, gs[i], rs[i])
# neighbour lists
Q = rs[:, :3].copy()
ids, d2, _, _ = ctx.knn(Q, Q, k=30)
t = O.Tree(Q)
oi, od = t.knn(Q, k=30)[:2]
print("knn ids equal", np.array_equal(ids, oi), "d2 equal", np.array_equal(d2, od))
print("labels equal", np.array_equal(g["labels"], r["labels"]), "out equal", np.array_equal(g["out"], r["out"]))
