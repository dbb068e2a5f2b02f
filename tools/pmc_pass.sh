#!/bin/bash
# One PMC pass per argument group ("NAME:CTR1,CTR2,..."), rocprofv3 --kernel-trace
# --pmc only, over an unpipelined bench run; summary in gpurun_out/pmc/summary_passes.txt.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --pmc 0 --no-stage-timing --frames-in-flight 1 ${PMC_EXTRA:-}"
for spec in "$@"; do
  n=${spec%%:*}; c=${spec#*:}; c=${c//,/ }
  rm -rf gpurun_out/pmc/$n
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $c -d gpurun_out/pmc/$n -o run --output-format csv -- $B > gpurun_out/pmc/$n.log 2>&1
  rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary_passes.txt 2>&1
grep -A1 "composite_kernel<0\|preprocess_kernel<3>\|bin_depth\|scan_dup\|rts_pass" gpurun_out/pmc/summary_passes.txt
