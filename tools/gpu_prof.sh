#!/bin/bash
# rocprofv3 kernel-trace stats of a short bench run (args: extra bench args).
# Writes gpurun_out/prof_<tag>/ and prints the kernel summary.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
TAG=${TAG:-x}
rm -rf gpurun_out/prof_$TAG
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_$TAG -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --pmc 0 "$@" > gpurun_out/prof_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || { tail -20 gpurun_out/prof_$TAG.log; exit $rc; }
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
    print(f'{r["Name"][:70]:70s} {int(r["Calls"]):5d} {float(r["AverageNs"])/1000:9.2f} us')
PY
