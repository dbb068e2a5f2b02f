#!/bin/bash
# Side-stream priority A/B (frames_in_flight 2) + a kernel trace at the default.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for p in 0 1 0 1; do
  GS_SIDE_PRIORITY=$p timeout -k 10 300 python bench.py --cpu-baseline 0 --traffic 0 --steps 60 --no-stage-timing \
    > gpurun_out/prio_$p.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/prio_$p.json'));print('prio',$p,d['ms_per_step'])"
done
rm -rf gpurun_out/ovlprof
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ovlprof -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --traffic 0 --no-stage-timing > gpurun_out/ovlprof.log 2>&1 || exit $?
echo done
