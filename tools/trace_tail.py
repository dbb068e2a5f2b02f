#!/usr/bin/env python3
"""Print the last N kernel dispatches of a rocprofv3 kernel trace (start, end,
duration in us relative to the first dispatch, queue, stream, kernel)."""
import csv
import sys

path = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 30
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
t0 = int(rows[0]["Start_Timestamp"])
for r in rows[-n:]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("gs::", "")[:30]
    print(f"{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:7.1f} q{r['Queue_Id']:>2} s{r['Stream_Id']} {name}")
