#!/bin/bash
# Round-6: does the composite's bin order change its HBM traffic?  FETCH_SIZE of the strip
# composite with the longest-first order (ab/lpt1, default) and row-major (ab/lpt0), and the
# frame times of both.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; export TMPDIR=/tmp; O=gpurun_out/lpt; mkdir -p $O
B="python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --pmc 0 --no-stage-timing --frames-in-flight 1 --settled-probe 0 --orbit-probe 0"
for v in lpt1 lpt0; do
  GSPLAT_LIB=$PWD/ab/$v.so timeout -s KILL 200 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $O/$v -o run --output-format csv -- $B > $O/$v.log 2>&1 || exit 1
  f=$(find $O/$v -name "*counter_collection.csv" | head -1)
  python - "$f" "$v" <<'PY'
import csv, sys, collections
s = collections.defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    if "composite_strip_kernel<0, 1>" in r["Kernel_Name"]:
        s[(r["Dispatch_Id"])].append(float(r["Counter_Value"]))
v = [sum(x) for x in s.values()]
print(sys.argv[2], "composite pass-1 FETCH_SIZE KB per launch (median of", len(v), "):", sorted(v)[len(v) // 2])
PY
done
for r in 1 2; do for v in lpt1 lpt0; do
  GSPLAT_LIB=$PWD/ab/$v.so timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 --steps 30 --settle 30 > $O/b_${v}_$r.json 2> $O/b_${v}_$r.err || exit 1
  python -c "import json;d=json.load(open('$O/b_${v}_$r.json'));print('$v r$r', d['ms_per_step'], 'orbit', d['orbit']['ms_per_step'], 'composite', round(d['stages']['composite']['ms'],4))"
done; done
