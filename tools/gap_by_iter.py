"""Gap between the update kernel and the next NN launch on the ICP stream, by iteration index of
the window (rocprofv3 kernel trace): python tools/gap_by_iter.py run_kernel_trace.csv"""
import collections
import csv
import re
import statistics
import sys

rows = list(csv.DictReader(open(sys.argv[1])))


def nm(r):
    m = re.search(r"(k_\w+)", r["Kernel_Name"])
    return m.group(1) if m else r["Kernel_Name"][:25]


q = [r["Queue_Id"] for r in rows if "k_icp_nn" in r["Kernel_Name"]][0]
rs = sorted([r for r in rows if r["Queue_Id"] == q], key=lambda r: int(r["Start_Timestamp"]))
it = 0
byit = collections.defaultdict(list)
for a, b in zip(rs, rs[1:]):
    if nm(a) == "k_active_list":
        it = 0
    if nm(a) == "k_icp_update_f" and nm(b) == "k_icp_nn":
        it += 1
        byit[it].append((int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1000)
for k in sorted(byit):
    v = byit[k]
    print(k, len(v), "median %.1f mean %.1f max %.1f us" % (statistics.median(v), statistics.mean(v), max(v)))
