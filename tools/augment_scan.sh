cd $GRAFT_REPO_ROOT
for a in "--B 4" "--B 16" "--B 1" "--B 4 --jitter none" "--B 16 --jitter none"; do
  timeout -k 10 120 python tools/augment_bench.py --no-cpu-baseline --iters 50 $a > gpurun_out/scan.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/scan.json'));print('$a', d['us_per_call'], d['value'], d['roofline']['frac'])"
done
