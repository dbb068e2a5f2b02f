#!/bin/bash
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out
for v in base lb0 ax0 fc0; do
  echo "== $v"
  if [ $v = base ]; then L=""; else L="GSPLAT_LIB=$PWD/ab/$v.so"; fi
  env $L timeout -k 10 120 python tools/dbg/retry_probe.py > gpurun_out/rp_$v.log 2>&1; rc=$?
  cat gpurun_out/rp_$v.log | tail -13; [ $rc -eq 0 ] || exit $rc
done
