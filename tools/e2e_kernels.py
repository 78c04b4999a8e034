#!/usr/bin/env python3
"""Dev: an e2e rocprofv3 trace (kernel + memory-copy csv of one run): the
library's kernels and the copies over the last `frac` of the run, their
totals by name and the busy time per stream.
   tools/e2e_kernels.py <dir with run_kernel_trace.csv> [frac]"""
import csv
import os
import re
import sys
from collections import defaultdict

d = sys.argv[1]
frac = float(sys.argv[2]) if len(sys.argv) > 2 else 0.6
ks = list(csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))))
cs = list(csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))))
ev = []
for r in ks:
    n = r["Kernel_Name"]
    n = n.replace("aqz::(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"\(.*$", "", n)
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "k:" + n, r["Stream_Id"]))
for r in cs:
    ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]),
               "c:" + r["Direction"].replace("MEMORY_COPY_", ""), "copy" + r["Stream_Id"]))
h2d = sorted(e for e in ev if e[2] == "c:HOST_TO_DEVICE")
t_end = max(e[1] for e in ev)
t_begin = h2d[int(len(h2d) * (1 - frac))][0]
span = (t_end - t_begin) / 1e6
tot = defaultdict(lambda: [0, 0.0])
st = defaultdict(float)
for s, e, n, sid in ev:
    if s < t_begin:
        continue
    tot[n][0] += 1
    tot[n][1] += (e - s) / 1e6
    st[sid] += (e - s) / 1e6
print(f"window {span:.1f} ms (last {frac:.0%} of the H2D copies)")
for n, (c, ms) in sorted(tot.items(), key=lambda x: -x[1][1])[:25]:
    print(f"  {n[:58]:58s} n {c:5d} total {ms:8.2f} ms avg {ms / c:7.3f}")
for k, ms in sorted(st.items()):
    print(f"  stream {k}: busy {ms:.1f} ms ({ms / span:.2f})")
