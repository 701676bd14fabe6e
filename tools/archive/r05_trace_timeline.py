"""Timeline of the resident pipeline from a rocprofv3 --kernel-trace CSV of
`bench.py` (3 batches in flight): per kernel class, the busy time and how
much of it overlaps other classes, over the timed region.
usage: python tools/r05_trace_timeline.py <trace dir> [last_n_dsmp]"""
import csv
import glob
import sys

d = sys.argv[1]
last = int(sys.argv[2]) if len(sys.argv) > 2 else 8
rows = []
for f in glob.glob(d + "/**/*kernel_trace.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        rows.append((r["Kernel_Name"].split("(")[0].split("<")[0], int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
rows.sort(key=lambda x: x[1])
ds = [r for r in rows if r[0] == "k_dsmp"]
if len(ds) < last + 1:
    sys.exit("only %d k_dsmp launches" % len(ds))
t0, t1 = ds[-last - 1][2], ds[-1][2]          # from the end of one DSM to the end of the last: `last` steps
win = [(n, max(a, t0), min(b, t1)) for n, a, b in rows if b > t0 and a < t1]


def union(iv):
    iv = sorted(iv)
    tot, cs, ce = 0, None, None
    for a, b in iv:
        if cs is None or a > ce:
            if cs is not None:
                tot += ce - cs
            cs, ce = a, b
        else:
            ce = max(ce, b)
    if cs is not None:
        tot += ce - cs
    return tot


span = t1 - t0
print("window: %d steps, %.3f ms per step" % (last, span / last / 1e6))
classes = sorted({n for n, _, _ in win})
for c in classes:
    iv = [(a, b) for n, a, b in win if n == c]
    print("%-10s launches %3d  busy %.3f ms/step  (sum of durations %.3f ms/step)"
          % (c, len(iv), union(iv) / last / 1e6, sum(b - a for a, b in iv) / last / 1e6))
dsm = [(a, b) for n, a, b in win if n in ("k_ai", "k_dsmp", "k_fin")]
front = [(a, b) for n, a, b in win if n in ("k_prep", "k_decomp")]
u_dsm, u_front, u_all = union(dsm), union(front), union(dsm + front)
print("DSM stage busy %.3f ms/step, fronts busy %.3f, either %.3f, overlap %.3f, idle %.3f"
      % (u_dsm / last / 1e6, u_front / last / 1e6, u_all / last / 1e6, (u_dsm + u_front - u_all) / last / 1e6,
         (span - u_all) / last / 1e6))
# k_dsmp back to back: gap between one k_dsmp's end and the next's start (negative = overlap)
dd = [r for r in win if r[0] == "k_dsmp"]
gaps = [(dd[i + 1][1] - dd[i][2]) / 1e3 for i in range(len(dd) - 1)]
print("k_dsmp start - previous k_dsmp end (us):", [round(g) for g in gaps])
