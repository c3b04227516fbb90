"""NN launches of a rocprofv3 kernel trace split by what ran beside them: the mean duration of
k_icp_nn dispatches that overlap another stream's kernel (by name) against those that overlap
nothing. Usage: python3 tools/nn_overlap.py run_kernel_trace.csv"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ev = [(int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0], r["Queue_Id"]) for r in rows]
nn = [e for e in ev if "k_icp_nn" in e[2]]
others = [e for e in ev if "k_icp_nn" not in e[2]]
others.sort()
by = defaultdict(list)
for s, t, name, q in nn:
    beside = {n for (a, b, n, qq) in others if qq != q and a < t and b > s}
    key = "alone" if not beside else ",".join(sorted(k[:22] for k in beside))[:110]
    by[key].append((t - s) / 1000.0)
for k, v in sorted(by.items(), key=lambda kv: -len(kv[1])):
    v.sort()
    print(f"{len(v):5d}  mean {sum(v)/len(v):7.1f} us  median {v[len(v)//2]:7.1f}  | {k}")
