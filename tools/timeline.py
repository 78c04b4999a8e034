"""Summarise a rocprofv3 kernel + memory-copy trace (tools/e2e_trace.sh):
per kernel name total/avg time, copy totals by direction, and the busy
fraction of the compute queue and of the copy engines over the traced
window's last N ms (the timed steps)."""
import csv
import sys
from collections import defaultdict

d = sys.argv[1]
tail_ms = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
ks = list(csv.DictReader(open(d + "/run_kernel_trace.csv")))
cs = list(csv.DictReader(open(d + "/run_memory_copy_trace.csv")))
end = max(int(r["End_Timestamp"]) for r in ks + cs)
start = end - tail_ms * 1e6 if tail_ms else min(int(r["Start_Timestamp"]) for r in ks + cs)


def clip(r):
    a, b = max(int(r["Start_Timestamp"]), start), int(r["End_Timestamp"])
    return (a, b) if b > a else None


def union(iv):
    iv = sorted(iv)
    tot, cur = 0, None
    for a, b in iv:
        if cur is None or a > cur[1]:
            if cur:
                tot += cur[1] - cur[0]
            cur = [a, b]
        else:
            cur[1] = max(cur[1], b)
    if cur:
        tot += cur[1] - cur[0]
    return tot


win = end - start
agg = defaultdict(lambda: [0, 0])
kiv = []
for r in ks:
    c = clip(r)
    if not c:
        continue
    agg[r["Kernel_Name"][:70]][0] += 1
    agg[r["Kernel_Name"][:70]][1] += c[1] - c[0]
    kiv.append(c)
print("window %.1f ms" % (win / 1e6))
for k, (n, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:14]:
    print("  %-70s n %4d total %8.2f ms (%4.1f%%)" % (k, n, t / 1e6, 100 * t / win))
print("kernels busy (union): %.1f%%" % (100 * union(kiv) / win))
cg = defaultdict(list)
cb = defaultdict(int)
for r in cs:
    c = clip(r)
    if not c:
        continue
    cg[r["Direction"]].append(c)
    cb[r["Direction"]] += int(r.get("Size", 0) or 0)
for k, iv in cg.items():
    u = union(iv)
    print("copies %-10s n %5d busy %.1f%%  %.2f GB  %.1f GB/s while busy" % (
        k, len(iv), 100 * u / win, cb[k] / 1e9, cb[k] / u if u else 0))
both = union(kiv + [x for v in cg.values() for x in v])
print("anything busy: %.1f%%" % (100 * both / win))
# per stream: busy fraction of the window and its heaviest kernels
ps = defaultdict(list)
pk = defaultdict(lambda: defaultdict(float))
for r in ks:
    c = clip(r)
    if not c:
        continue
    sid = r.get("Stream_Id", r.get("Queue_Id", "?"))
    ps[sid].append(c)
    pk[sid][r["Kernel_Name"][:40]] += (c[1] - c[0]) / 1e6
for sid, iv in sorted(ps.items(), key=lambda x: -union(x[1])):
    top = sorted(pk[sid].items(), key=lambda x: -x[1])[:4]
    print("stream %-4s busy %5.1f%%  " % (sid, 100 * union(iv) / win) +
          ", ".join("%s %.2f ms" % (k, t) for k, t in top))
