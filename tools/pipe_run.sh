cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
for fif in 1 2 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --traffic 0 --steps 30 --frames-in-flight $fif > gpurun_out/b_$fif.json 2> gpurun_out/b_$fif.err
  rc=$?; echo "fif=$fif rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/b_$fif.json'));print(d['ms_per_step'], d['value'], d['timed_kernel_ms'])")"; [ $rc -eq 0 ] || exit $rc
done
