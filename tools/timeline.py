"""Per-stream timeline of one C2 window from a rocprofv3 kernel trace (run_kernel_trace.csv):
python3 tools/timeline.py TRACE.csv [window index] -- prints each kernel's start / end (us) from
the window's k_seq_ref_points, its stream and duration, so the critical chain and what runs
beside it are visible."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
w = int(sys.argv[2]) if len(sys.argv) > 2 else 20
for r in rows:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
refs = [r for r in rows if "k_seq_ref_points" in r["Kernel_Name"]]
t0 = refs[w]["s"]
t1 = refs[w + 1]["s"]
short = lambda n: re.sub(r"\(.*", "", re.sub(r"aicp::|\(anonymous namespace\)::|void |rocprim::ROCPRIM_\d+_NS::detail::", "", n))[:38]
for r in rows:
    if r["e"] < t0 - 20000 or r["s"] > t1:
        continue
    print("%8.1f %8.1f  q%-3s %6.1f  %s" % ((r["s"] - t0) / 1e3, (r["e"] - t0) / 1e3, r["Queue_Id"],
                                          (r["e"] - r["s"]) / 1e3, short(r["Kernel_Name"])))
print("period %.1f us" % ((t1 - t0) / 1e3))
