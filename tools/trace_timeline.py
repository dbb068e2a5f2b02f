#!/usr/bin/env python3
"""Timeline of a rocprofv3 --kernel-trace CSV: per kernel start/end (us,
relative), queue, and per-frame phases (preprocess, chain, composite) with
their overlap.  python tools/trace_timeline.py <run_kernel_trace.csv> [frames]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
nf = int(sys.argv[2]) if len(sys.argv) > 2 else 6
ks = []
for r in rows:
    name = r.get("Kernel_Name", "")
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    ks.append((s, e, name.split("(")[0].replace("void ", "").replace("gs::", ""), r.get("Queue_Id", r.get("Stream_Id", "?"))))
ks.sort()
t0 = ks[0][0]
# last frames
pre = [k for k in ks if k[2].startswith("preprocess")]
start = pre[-nf - 1][0] if len(pre) > nf else t0
for s, e, n, q in ks:
    if s >= start:
        print(f"{(s - start) / 1e3:9.1f} {(e - start) / 1e3:9.1f} {(e - s) / 1e3:7.1f}  q{q:>3}  {n[:40]}")
comp = [k for k in ks if k[2].startswith("composite")]
if len(comp) > 2:
    ends = [c[1] for c in comp[-nf:]]
    per = [(ends[i + 1] - ends[i]) / 1e3 for i in range(len(ends) - 1)]
    print("composite-end to composite-end (us):", " ".join(f"{p:.1f}" for p in per))
