#!/bin/bash
# Group (gs_create_sharded) GPU tests, then ingest timings at 6M and (disk permitting) 50M.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=${TMPDIR:-/tmp}
timeout -k 10 600 python -u -m pytest tests/test_gpu_group.py tests/test_ingest.py -v --timeout 300 --timeout-method thread > gpurun_out/pytest_group.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|SKIP|passed|failed" gpurun_out/pytest_group.log | tail -30; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
df -h "$TMPDIR" | tail -1
timeout -k 10 600 python tools/ingest_bench.py --splats 6000000 > gpurun_out/ingest_6m.json; rc=$?; cat gpurun_out/ingest_6m.json; [ $rc -eq 0 ] || exit $rc
avail=$(df --output=avail -k "$TMPDIR" | tail -1)
if [ "$avail" -gt 31000000 ]; then
  timeout -k 10 900 python tools/ingest_bench.py --splats 50000000 > gpurun_out/ingest_50m.json; rc=$?; cat gpurun_out/ingest_50m.json; [ $rc -eq 0 ] || exit $rc
else echo "skip 50M: $avail KB free"; fi
