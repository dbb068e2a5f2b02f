cd "${GRAFT_REPO_ROOT:-/root/repo}"; mkdir -p gpurun_out; export TMPDIR=/tmp
for r in 1 2 3; do
  for a in "--steps 20 --warmup 5" "--steps 100 --warmup 5" "--steps 20 --warmup 50"; do
    timeout -k 10 300 python bench.py --cpu-baseline 0 --pmc 0 $a > gpurun_out/st.json 2>/dev/null || exit 1
    echo "$a: $(python -c "import json;print(json.load(open('gpurun_out/st.json'))['ms_per_step'])")"
  done
done
