#!/bin/bash
# Round-6: the resident strip composite (GS_STRIP_PERSIST).
# Its parity tests on ab/${TESTV:-sp1}.so, then an A/B of VARIANTS at 1080p, 4K, 50M
# (sp0 = the default build, sp1 = resident 2048 workgroups, sp1k = 1024).
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
GSPLAT_LIB=$PWD/ab/${TESTV:-sp1}.so timeout -k 10 700 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_depth_split.py tests/test_gpu_configs.py -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/sp_pt.log 2>&1
rc=$?; tail -2 gpurun_out/sp_pt.log; [ $rc -eq 0 ] || exit $rc
NOTEST=1 VARIANTS="${VARIANTS:-sp0 sp1 sp1k}" CFGS="${CFGS:-1080p 4k 50m}" bash tools/gpu_r06_s2.sh
