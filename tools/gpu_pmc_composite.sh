#!/bin/bash
# Memory-path PMC passes for the composite (TLB, TCP, TA, TD), one rocprofv3 run per group.
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out/pmc; export TMPDIR=/tmp
B="python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --pmc 0 --no-stage-timing --frames-in-flight 1"
run() { n=$1; shift; rm -rf gpurun_out/pmc/$n; timeout -k 10 200 rocprofv3 --kernel-trace --pmc "$@" -d gpurun_out/pmc/$n -o run --output-format csv -- $B > gpurun_out/pmc/$n.log 2>&1; rc=$?; echo "$n rc=$rc"; [ $rc -eq 0 ] || exit $rc; }
run tlb TCP_UTCL1_REQUEST_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_STALL_INFLIGHT_MAX_sum TCP_UTCL1_STALL_MULTI_MISS_sum
run tcp TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum
run ta1 TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum
run ta2 TA_DATA_STALLED_BY_TC_CYCLES_sum TA_FLAT_READ_WAVEFRONTS_sum
run td TD_TD_BUSY_sum TD_TC_STALL_sum
run tlb2 TCP_UTCL1_THRASHING_STALL_sum TCP_UTCL1_TRANSLATION_MISS_UNDER_MISS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_TCC_READ_REQ_LATENCY_sum
run grbm GRBM_GUI_ACTIVE GRBM_COUNT
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary_mem.txt 2>&1
grep -A1 "composite_kernel<0\|preprocess_kernel<3>" gpurun_out/pmc/summary_mem.txt
