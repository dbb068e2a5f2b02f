"""Summarise rocprofv3 --pmc CSVs: mean counter value per kernel (per dispatch)."""
import csv
import sys
from collections import defaultdict
from pathlib import Path

root = Path(sys.argv[1])
vals = defaultdict(lambda: defaultdict(list))
for f in root.rglob("*counter_collection.csv"):
    with open(f) as fh:
        for row in csv.DictReader(fh):
            k = row.get("Kernel_Name", "?").split("(")[0].replace("void ", "")
            vals[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
for k in sorted(vals):
    cs = vals[k]
    parts = [f"{c}={sum(v)/len(v):.4g}" for c, v in sorted(cs.items())]
    print(k)
    print("   " + "  ".join(parts))
