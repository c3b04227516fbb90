"""Per-stream timeline of one window of the C2 stream from a rocprofv3 kernel trace:
python tools/timeline_seq.py <run_kernel_trace.csv> [run index] [window index]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
run = int(sys.argv[2]) if len(sys.argv) > 2 else 3
win = int(sys.argv[3]) if len(sys.argv) > 3 else 6
for r in rows:
    r["s"] = int(r["Start_Timestamp"])
    r["e"] = int(r["End_Timestamp"])
    nm = r["Kernel_Name"].replace("(anonymous namespace)::", "")
    base = nm.split("(")[0]
    if "rocprim" in base:
        base = "rocprim::" + ("init_lookback" if "init_lookback" in nm else "scan" if "scan" in nm else
                              "sort" if "sort" in nm else "other")
    r["n"] = base.replace("aicp::", "").replace("void ", "")[-40:]
rows.sort(key=lambda r: r["s"])
fin = [r for r in rows if "k_finalize" in r["n"]]
# 13 windows per run; run boundaries: finalize index
per = 13
f = fin[run * per:(run + 1) * per]
t0 = f[win - 1]["e"] if win > 0 else None
t1 = f[win]["e"]
print("window %d of run %d: %.1f us between finalizes" % (win, run, (t1 - t0) / 1e3))
span = [r for r in rows if t0 <= r["s"] <= t1]
streams = {}
for r in span:
    streams.setdefault(r["Stream_Id"], []).append(r)
for sid, rs in sorted(streams.items()):
    busy = sum(r["e"] - r["s"] for r in rs)
    print("stream %s: %d kernels, busy %.1f us, first %.1f last %.1f" % (sid, len(rs), busy / 1e3, (rs[0]["s"] - t0) / 1e3,
                                                                      (rs[-1]["e"] - t0) / 1e3))
    agg = {}
    for r in rs:
        a = agg.setdefault(r["n"], [0, 0])
        a[0] += 1
        a[1] += r["e"] - r["s"]
    for n, (c, d) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
        print("   %-42s %4d  %8.1f us" % (n, c, d / 1e3))
