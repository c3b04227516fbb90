#!/usr/bin/env python3
"""Timeline of the last batch run in a rocprofv3 kernel trace: python tools/timeline.py TRACE.csv [RUN]

A run starts at each k_init_state launch that follows a gap; prints every kernel of run RUN
(default: the last) with its stream, start offset and duration in microseconds, then the
per-stream busy time and the gaps (>20 us) on each stream."""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
    r["n"] = r["Kernel_Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("aicp::", "")
    if "rocprim" in r["n"]:
        r["n"] = "rocprim::" + ("scan" if "scan" in r["Kernel_Name"] else "sort" if "sort" in r["Kernel_Name"] else "other")
rows.sort(key=lambda r: r["s"])
starts = [i for i, r in enumerate(rows) if r["n"].startswith("k_init_state") and (i == 0 or rows[i - 1]["n"] != r["n"])]
runs = [rows[a:b] for a, b in zip(starts, starts[1:] + [len(rows)])]
want = int(sys.argv[2]) if len(sys.argv) > 2 else -1
run = runs[want]
# the init_state of the reference stream belongs to the run too
t0 = run[0]["s"]
print(f"{len(runs)} runs; run {want}: {len(run)} kernels, span {(max(r['e'] for r in run) - t0) / 1e3:.1f} us")
last_end = {}
for r in run:
    q = r["Queue_Id"]
    gap = (r["s"] - last_end[q]) / 1e3 if q in last_end else 0
    last_end[q] = r["e"]
    mark = f"  gap {gap:7.1f}" if gap > 20 else ""
    print(f"q{q:>2s} {(r['s'] - t0) / 1e3:9.1f} {(r['e'] - r['s']) / 1e3:8.1f}  {r['n'][:70]}{mark}")
