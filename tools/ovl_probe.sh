#!/bin/bash
# Frames-in-flight probe: bench at fif 1 and 2 (no stage timing), then a
# kernel trace of a short fif-2 run to see the composite/projection overlap.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for f in 1 2 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --traffic 0 --steps 60 --no-stage-timing --frames-in-flight $f \
    > gpurun_out/ovl_f$f.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/ovl_f$f.json'));print('fif',$f,d['ms_per_step'])"
done
rm -rf gpurun_out/ovlprof
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/ovlprof -o run --output-format csv -- \
  python bench.py --steps 10 --warmup 3 --cpu-baseline 0 --traffic 0 --no-stage-timing > gpurun_out/ovlprof.log 2>&1 || exit $?
echo done
