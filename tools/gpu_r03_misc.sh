cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "shard or slab or group or rows or band or config4 or config5 or bench" --timeout 300 --timeout-method thread > gpurun_out/shard_tests.log 2>&1; rc=$?; tail -2 gpurun_out/shard_tests.log; [ $rc -eq 0 ] || exit $rc
rm -rf gpurun_out/rt && timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/rt -o run --output-format csv -- python tools/rows_trace.py > gpurun_out/rt.log 2>&1 || exit 1
python tools/rows_trace.py --analyze $(find gpurun_out/rt -name "*kernel_trace.csv" | head -1) > gpurun_out/rt.txt; head -8 gpurun_out/rt.txt
GSPLAT_LIB=ab/cnt.so timeout -k 10 300 python tools/composite_counters.py > gpurun_out/cnt.txt 2>&1 || exit 1; tail -3 gpurun_out/cnt.txt
rm -rf gpurun_out/tcc && timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_REQ_sum -d gpurun_out/tcc -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --pmc 0 --no-stage-timing --frames-in-flight 1 > gpurun_out/tcc.log 2>&1 || exit 1
python - <<'PY'
import csv, glob, collections
f = glob.glob("gpurun_out/tcc/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")[:40]
    acc[(k, r["Counter_Name"])].append(float(r["Counter_Value"]))
for (k, c), v in sorted(acc.items()):
    if "composite" in k or "preprocess" in k or "rts_pass" in k or "duplicate" in k:
        print(f"{k:40s} {c:14s} {sum(v)/len(v):.4g}")
PY
