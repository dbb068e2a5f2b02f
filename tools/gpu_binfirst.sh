cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "bin_first or sorted_pairs or config1 or 1080p" --timeout 120 --timeout-method thread > gpurun_out/pt_binfirst.log 2>&1
rc=$?; tail -15 gpurun_out/pt_binfirst.log; echo "pytest rc=$rc"
[ $rc -eq 0 ] || exit $rc
for b in depth bin; do
  GS_BINNING=$b timeout -k 10 300 python bench.py --cpu-baseline 0 --traffic 0 > gpurun_out/bench_$b.json 2> gpurun_out/bench_$b.err
  rc=$?; echo "$b rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/bench_$b.json'));print('$b', d['ms_per_step'], {k:round(v['ms'],4) for k,v in d['stages'].items()})"
done
