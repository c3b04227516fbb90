"""Prefilter GPU vs oracle cluster diagnostics (not part of the product)."""
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
gl, rl = g["labels"], r["labels"]
print("n_clusters", g["n_clusters"], r["n_clusters"], "out", len(g["out"]), len(r["out"]))
print("gpu sizes", np.bincount(gl[gl >= 0]), "(-1:", (gl < 0).sum(), ")")
print("ora sizes", np.bincount(rl[rl >= 0]), "(-1:", (rl < 0).sum(), ")")
pairs = {}
for a, b in zip(gl, rl):
    pairs[(int(a), int(b))] = pairs.get((int(a), int(b)), 0) + 1
print("contingency (gpu, oracle): count", sorted(pairs.items()))
print("out rows equal to sampled rows:", np.isin(g["out"].view("V12"), g["sampled"][:, :3].copy().view("V12")).sum())
