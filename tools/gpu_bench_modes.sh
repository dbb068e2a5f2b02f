# bench.py across its options (each must produce one JSON line): modes, one frame in flight, orbit at 1M.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for a in "--mode live50" "--mode mlab" "--frames-in-flight 1" "--config 1m --camera orbit" "--config 4k --camera orbit --steps 30"; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 $a > gpurun_out/bm.json 2> gpurun_out/bm.err || { echo "FAIL $a"; tail -5 gpurun_out/bm.err; exit 1; }
  python3 -c "import json;d=json.load(open('gpurun_out/bm.json'));print('$a', d['ms_per_step'], d['value'], d['config']['binning'], d['config']['pairs'], d['config']['visible'])"
done
