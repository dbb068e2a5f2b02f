#!/bin/bash
# A/B with parity: the composite-path parity tests against each ab/<name>.so
# named in AB_PARITY (default: every variant but base), then tools/ab.sh twice.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for so in ab/*.so; do
  v=$(basename "$so" .so); [ "$v" = base ] && continue
  GSPLAT_LIB=$PWD/$so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -m gpu \
    -k "${AB_TESTS:-1080p or config1 or cap_parity or virtual_slabs}" --timeout 120 --timeout-method thread \
    > gpurun_out/pt_$v.log 2>&1
  rc=$?; echo "$v parity rc=$rc $(tail -1 gpurun_out/pt_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
bash tools/ab.sh && bash tools/ab.sh
