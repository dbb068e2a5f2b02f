#!/bin/bash
# A/B of pipeline schedules: each entry of CFGS is a comma-separated env list
# ("-" = defaults), e.g. CFGS="- GS_PIPE_SCHED=pc,GS_PRE_GRID=4".  Bench each ROUNDS
# times interleaved, optional PARITY (pytest -k expr, under PARITY_ENV or the defaults), then a
# kernel-trace timeline of each config in TL (indices into CFGS).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
read -ra C <<< "${CFGS:--}"
envof() { [ "$1" = "-" ] && return; echo "$1" | tr ',' ' '; }
if [ -n "$PARITY" ]; then
  env $(envof "${PARITY_ENV:--}") timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "$PARITY" --timeout 200 --timeout-method thread > gpurun_out/sch_parity.log 2>&1
  rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/sch_parity.log)"; [ $rc -eq 0 ] || exit $rc
fi
for r in $(seq ${ROUNDS:-2}); do
  for i in "${!C[@]}"; do
    env $(envof "${C[$i]}") timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 ${BENCH_ARGS} > gpurun_out/sch_${i}_$r.json 2> gpurun_out/sch_${i}_$r.err
    rc=$?
    echo "${C[$i]} r$r rc=$rc $(python -c "import json;d=json.load(open('gpurun_out/sch_${i}_$r.json'));print(d['ms_per_step'], 'sa', d['standalone_kernel_ms'], 'timed', d['timed_kernel_ms'])" 2>/dev/null)"
    [ $rc -eq 0 ] || { tail -3 gpurun_out/sch_${i}_$r.err; exit $rc; }
  done
done
for i in ${TL}; do
  rm -rf gpurun_out/tl_$i
  env $(envof "${C[$i]}") timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/tl_$i -o run --output-format csv -- python bench.py --steps 20 --warmup 3 --cpu-baseline 0 --pmc 0 --no-stage-timing ${BENCH_ARGS} > gpurun_out/tl_$i.log 2>&1; rc=$?; echo "tl ${C[$i]} rc=$rc"
  [ $rc -eq 0 ] || exit $rc
  f=$(find gpurun_out/tl_$i -name "*kernel_trace.csv" | head -1); python tools/trace_timeline.py $f 3 > gpurun_out/tl_$i.txt; tail -${TL_LINES:-16} gpurun_out/tl_$i.txt
done
