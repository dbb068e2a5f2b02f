#!/bin/bash
# Round-6 session 9: the -m gpu suite on HEAD; PMC of the radix passes with (pair1) and without
# (pair0) (key, value) pair staging, at 1080p and 50M (unpipelined frames).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/s9_pt.log 2>&1
rc=$?; tail -2 gpurun_out/s9_pt.log; [ $rc -eq 0 ] || exit $rc
for cfg in 1080p 50m; do
  STEPS=pmc VARIANTS="pair1 pair0" BENCH_ARGS="--config $cfg" PMC_TRAFFIC="" bash tools/gpu_r05.sh > /dev/null || exit 1
  for v in pair1 pair0; do cp gpurun_out/pmc_$v/summary.txt gpurun_out/s9_pmc_${cfg}_$v.txt; echo "== $cfg $v"; grep -A1 "rts_pass\|bin_depth_sort" gpurun_out/pmc_$v/summary.txt | python3 -c "
import sys,re
lines=sys.stdin.read().split('\n')
for i,l in enumerate(lines):
    if l.startswith('gs::'):
        d=dict(re.findall(r'(\w+)=([\d.e+]+)', lines[i+1]))
        c=float(d.get('SQ_LDS_BANK_CONFLICT',0)); a=float(d.get('SQ_LDS_IDX_ACTIVE',1)); w=float(d.get('SQ_WAIT_INST_ANY',0)); wc=float(d.get('SQ_WAVE_CYCLES',1)); lds=float(d.get('SQ_INSTS_LDS',0))
        print(l[:60], 'conflict/active %.3f'%(c/a), 'lds_insts %.3g'%lds, 'conflict %.3g'%c, 'wait_inst %.2f'%(w/wc))
"; done
done
