"""Short per-kernel summary of a rocprofv3 kernel_stats.csv: calls, average us, total ms, share."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
for r in rows[: int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    n = r["Name"]
    n = re.sub(r"rocprim::ROCPRIM_\w+::detail::trampoline_kernel<rocprim::ROCPRIM_\w+::detail::wrapped_(\w+).*", r"rocprim:\1", n)
    n = n.replace("(anonymous namespace)::", "").replace("aicp::", "")
    n = re.sub(r"\(.*", "", n)
    print("%-40s %7d %10.2f %10.2f %6.2f%%" % (n[:40], int(r["Calls"]), float(r["AverageNs"]) / 1e3,
                                             float(r["TotalDurationNs"]) / 1e6, 100 * float(r["TotalDurationNs"]) / tot))
print("total kernel ms %.2f" % (tot / 1e6))
