cd "${GRAFT_REPO_ROOT:-/root/repo}"
mkdir -p gpurun_out
for cfg in "6000000 3840 2160" "50000000 3840 2160"; do
  set -- $cfg
  timeout -k 10 600 python bench.py --cpu-baseline 0 --traffic 0 --steps 10 --warmup 3 --splats $1 --width $2 --height $3 > gpurun_out/scale_$1_$2.json 2> gpurun_out/scale_$1_$2.err
  rc=$?; echo "cfg=$cfg rc=$rc"; tail -2 gpurun_out/scale_$1_$2.err; [ $rc -eq 0 ] || exit $rc
  python -c "import json;d=json.load(open('gpurun_out/scale_$1_$2.json'));print(d['ms_per_step'], d['value'], d['config']['pairs'], d['roofline']['kernel'], d['roofline']['frac'], {k:round(v['ms'],3) for k,v in d['stages'].items()})"
done
