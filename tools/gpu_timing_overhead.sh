# Does the dispatch-packet event timing (stage_timing 2) cost the timed frames anything?
cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for a in "" "--no-stage-timing"; do
    timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 $a > gpurun_out/to.json 2>/dev/null || exit 1
    echo "[$a] r$r $(python -c "import json;print(json.load(open('gpurun_out/to.json'))['ms_per_step'])")"
  done
done
