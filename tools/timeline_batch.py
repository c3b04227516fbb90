"""Per-queue phases of one batched call (C5 / C3 batched / C4) from a rocprofv3 kernel trace:
python3 tools/timeline_batch.py TRACE.csv [call index] -- a call starts at a k_tr_zero that
follows a gap of > 5 ms without kernels; consecutive kernels of one queue are merged into phases
by name class (tree, knn, normals, overlap, icp, other), printed with start / end (ms) from the
call's first kernel and their busy time, so the critical chain of the call is visible."""
import csv
import re
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
ci = int(sys.argv[2]) if len(sys.argv) > 2 else 1
for r in rows:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
rows.sort(key=lambda r: r["s"])
# calls: kernels separated by > 5 ms of idle device
calls, cur, last = [], [], None
for r in rows:
    if last is not None and r["s"] - last > 5e6:
        calls.append(cur)
        cur = []
    cur.append(r)
    last = max(last or 0, r["e"])
calls.append(cur)
call = calls[ci]
short = lambda n: re.sub(r"\(.*", "", re.sub(r"aicp::|\(anonymous namespace\)::|void |rocprim::ROCPRIM_\d+_NS::detail::", "", n))[:24]
t0 = call[0]["s"]


def cls(n):
    n = n.lower()
    if "k_icp" in n or "k_sel" in n or "k_active" in n or "k_solve" in n or "k_finalize" in n or "k_prepare" in n:
        return "icp"
    if "knn" in n:
        return "knn"
    if "normals" in n or "inv_perm" in n or "scatter_normals" in n:
        return "normals"
    if "k_ovl" in n or "radix" in n or "onesweep" in n or "morton" in n:
        return "overlap/sort"
    if "k_tr" in n or "k_tl" in n:
        return "tree"
    return "other"


print("call %d of %d: %.2f ms, %d kernels" % (ci, len(calls), (max(r["e"] for r in call) - t0) / 1e6, len(call)))
for q in sorted({r["Queue_Id"] for r in call}):
    ks = [r for r in call if r["Queue_Id"] == q]
    ph = []
    for r in ks:
        c = cls(r["Kernel_Name"])
        if ph and ph[-1][0] == c:
            ph[-1][2] = r["e"]
            ph[-1][3] += r["e"] - r["s"]
            ph[-1][4] += 1
            nm = short(r["Kernel_Name"])
            ph[-1][5][nm] = ph[-1][5].get(nm, 0) + (r["e"] - r["s"])
        else:
            nm = short(r["Kernel_Name"])
            ph.append([c, r["s"], r["e"], r["e"] - r["s"], 1, {nm: r["e"] - r["s"]}])
    print("queue %s:" % q)
    for c, s, e, busy, n, top in ph:
        tops = sorted(top.items(), key=lambda kv: -kv[1])[:3]
        print("  %-13s %8.2f %8.2f  busy %7.2f ms  %4d kernels  %s" % (
            c, (s - t0) / 1e6, (e - t0) / 1e6, busy / 1e6, n,
            ", ".join("%s %.1f" % (k, v / 1e6) for k, v in tops)))
