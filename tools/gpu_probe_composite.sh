cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
GSPLAT_LIB=ab/ct.so timeout -k 10 300 python tools/composite_counters.py > gpurun_out/ct.txt 2>&1; rc=$?; cat gpurun_out/ct.txt; [ $rc -eq 0 ] || exit $rc
GSPLAT_LIB=ab/cnt.so timeout -k 10 300 python tools/composite_counters.py > gpurun_out/cnt.txt 2>&1; rc=$?; cat gpurun_out/cnt.txt; [ $rc -eq 0 ] || exit $rc
mkdir -p gpurun_out/pmc
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU -d gpurun_out/pmc/sq1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --pmc 0 --no-stage-timing --frames-in-flight 1 > gpurun_out/pmc/sq1.log 2>&1; echo "sq1 rc=$?"
timeout -k 10 300 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE -d gpurun_out/pmc/sq2 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --cpu-baseline 0 --pmc 0 --no-stage-timing --frames-in-flight 1 > gpurun_out/pmc/sq2.log 2>&1; echo "sq2 rc=$?"
python tools/pmc_summary.py gpurun_out/pmc > gpurun_out/pmc/summary.txt 2>&1; grep -A1 "composite_kernel<0" gpurun_out/pmc/summary.txt
