#!/bin/bash
# kernel stats of band frames (tools/band_probe.py, world 2, 1080p)
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/btl -o run --output-format csv -- python tools/band_probe.py --worlds 2 --frames 20 > gpurun_out/btl.log 2>&1 || exit 1
f=$(find gpurun_out/btl -name "*kernel_stats.csv" | head -1)
python -c "
import csv,sys
rows=list(csv.DictReader(open('$f')))
for r in rows[:16]: print(r['Name'][:70], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
