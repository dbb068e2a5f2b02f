#!/bin/bash
# Multi-GPU evidence on one GPU (round 3): shard/band/group/bench-rank GPU tests, the
# rows probe at 1080p and 4K, the band probe, and one rank's row-frame kernel trace.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu -k "shard or slab or group or rows or band or config4 or config5 or bench" --timeout 300 --timeout-method thread > gpurun_out/mg_tests.log 2>&1; rc=$?; tail -1 gpurun_out/mg_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python tools/rows_probe.py > gpurun_out/rows_probe_1080p.json 2> gpurun_out/rows_probe_1080p.err || exit 1
timeout -k 10 400 python tools/rows_probe.py --width 3840 --height 2160 > gpurun_out/rows_probe_4k.json 2> gpurun_out/rows_probe_4k.err || exit 1
timeout -k 10 400 python tools/band_probe.py > gpurun_out/band_probe_1080p.json 2> gpurun_out/band_probe_1080p.err || exit 1
grep -h "probe\]" gpurun_out/rows_probe_1080p.err gpurun_out/rows_probe_4k.err gpurun_out/band_probe_1080p.err
rm -rf gpurun_out/rt && timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/rt -o run --output-format csv -- python tools/rows_trace.py > gpurun_out/rt.log 2>&1 || exit 1
python tools/rows_trace.py --analyze $(find gpurun_out/rt -name "*kernel_trace.csv" | head -1) > gpurun_out/rows_trace_world8.txt
