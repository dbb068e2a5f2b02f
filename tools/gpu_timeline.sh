cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
rm -rf gpurun_out/tl
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --pmc 0 --no-stage-timing ${TL_ARGS} > gpurun_out/tl.log 2>&1; rc=$?; echo rc=$rc
f=$(find gpurun_out/tl -name "*kernel_trace.csv" | head -1); python tools/trace_timeline.py $f 4 > gpurun_out/tl.txt; tail -45 gpurun_out/tl.txt
