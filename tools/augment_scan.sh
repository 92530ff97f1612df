#!/bin/bash
# A/B scan of the augment micro-bench (batch size, jitter on/off, vertical-pass vector width).
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for a in "--B 4" "--B 16" "--B 4 --jitter none" "VEC1 --B 4" "VEC1 --B 16"; do
  env=""; args=$a
  case $a in VEC1*) env="PSFM_AUGMENT_VEC=1"; args=${a#VEC1 };; esac
  env $env timeout -k 10 120 python tools/augment_bench.py --no-cpu-baseline --iters 50 $args > gpurun_out/scan.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/scan.json'));print('$a', d['us_per_call'], d['value'], d['roofline']['frac'])"
done
