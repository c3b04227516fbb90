#!/usr/bin/env python3
"""Print a rocprofv3 kernel_stats.csv as a per-run table: python tools/kstats.py STATS.csv RUNS"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
runs = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"{'kernel':60s} {'calls/run':>9s} {'avg us':>9s} {'ms/run':>8s} {'%':>6s}")
for r in rows:
    name = r["Name"].replace("(anonymous namespace)::", "").split("(")[0].replace("void ", "").replace("aicp::", "")[:60]
    t = float(r["TotalDurationNs"])
    print(f"{name:60s} {float(r['Calls']) / runs:9.1f} {float(r['AverageNs']) / 1e3:9.1f} {t / 1e6 / runs:8.3f} {100 * t / tot:6.2f}")
print(f"{'total':60s} {'':9s} {'':9s} {tot / 1e6 / runs:8.3f}")
