# The driver's own bench command (BENCH_r02.json: --gpus 1 --steps 20 --warmup 5), twice, timed by wall clock,
# plus the 2-rank bench rehearsal test.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2; do
  t0=$(date +%s.%N)
  timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/drv_$r.json 2> gpurun_out/drv_$r.err || exit 1
  t1=$(date +%s.%N)
  python3 -c "import json;d=json.load(open('gpurun_out/drv_$r.json'));print('run $r', d['ms_per_step'], d['value'], d['settle'], 'wall_s', round($t1-$t0,1))"
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_ranks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/drv_ranks.log 2>&1; rc=$?
echo "ranks rc=$rc $(tail -1 gpurun_out/drv_ranks.log)"; exit $rc
