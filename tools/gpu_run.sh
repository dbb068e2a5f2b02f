#!/bin/bash
# One GPU session: parity tests -> bench -> rocprofv3 kernel stats.
# Each GPU step has its own time limit; a crash/timeout/fault stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS="${STEPS:-tests bench prof}"
stop_if_bad() {  # rc 0 = pass, 1 = test failure (not a fault) -> continue
  rc=$1; what=$2
  echo "$what rc=$rc"
  if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $what (rc=$rc)"; exit "$rc"; fi
}
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 900 python -m pytest tests -x -q -m gpu ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
      stop_if_bad $? pytest; tail -30 gpurun_out/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      stop_if_bad $? smoke; tail -5 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
      stop_if_bad $? bench; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python bench.py --steps 10 --warmup 3 --cpu-baseline 0 ${PROF_ARGS} > gpurun_out/prof.log 2>&1
      stop_if_bad $? rocprof; tail -3 gpurun_out/prof.log
      find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \; | head -40 ;;
  esac
done
