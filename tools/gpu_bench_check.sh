# Bench JSON sanity after bench.py changes: the driver's command, the default command, the 2-rank rehearsal test.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bc_drv.json 2> gpurun_out/bc_drv.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bc_drv.json'));print('driver cmd', d['ms_per_step'], d['timed_kernel_ms'], d['timed_kernel_note'], d['standalone_kernel_ms'], d['roofline']['frac'], d['roofline']['traffic'])"
timeout -k 10 600 python3 bench.py --cpu-baseline 0 > gpurun_out/bc_def.json 2> gpurun_out/bc_def.err || exit 1
python3 -c "import json;d=json.load(open('gpurun_out/bc_def.json'));print('default', d['ms_per_step'], d['timed_kernel_ms'], d['standalone_kernel_ms'])"
timeout -k 10 400 python -u -m pytest tests/test_gpu_bench_ranks.py -x -q --timeout 300 --timeout-method thread > gpurun_out/bc_ranks.log 2>&1; rc=$?
echo "ranks rc=$rc $(tail -1 gpurun_out/bc_ranks.log)"; exit $rc
