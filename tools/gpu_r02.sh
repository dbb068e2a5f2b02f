#!/bin/bash
# Round-2 GPU session: parity tests -> bench -> rocprofv3 kernel stats.
# Every GPU step has its own time limit; anything but pass/test-failure stops the script.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
STEPS="${STEPS:-tests bench prof}"
stop_if_bad() { rc=$1; echo "$2 rc=$rc"; if [ "$rc" -ne 0 ] && [ "$rc" -ne 1 ]; then echo "stopping after $2"; exit "$rc"; fi; }
for s in $STEPS; do
  case $s in
    tests)
      timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread ${PYTEST_ARGS} > gpurun_out/pytest_gpu.log 2>&1
      stop_if_bad $? pytest; grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_gpu.log | tail -60 ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
      stop_if_bad $? smoke; tail -3 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.json 2> gpurun_out/bench.err
      stop_if_bad $? bench; cat gpurun_out/bench.json; tail -5 gpurun_out/bench.err ;;
    prof)
      rm -rf gpurun_out/prof
      timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
        python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --pmc 0 ${PROF_ARGS} > gpurun_out/prof.log 2>&1
      stop_if_bad $? rocprof; tail -3 gpurun_out/prof.log
      find gpurun_out/prof -name "*kernel_stats.csv" -exec cat {} \; | cut -c1-200 | head -30 ;;
  esac
done
