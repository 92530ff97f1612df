#!/bin/bash
# A/B scan of the augment micro-bench: horizontal-pass workgroup size and vertical-pass vector
# width (env knobs of psfm_augment.hip), batch size.
cd ${GRAFT_REPO_ROOT:-$(pwd)}
for v in "X=1" "PSFM_AUGMENT_NTH=320" "PSFM_AUGMENT_NTH=640" "PSFM_AUGMENT_NTH=128" "X=1 --B 16" "PSFM_AUGMENT_NTH=320 --B 16"; do
  env=${v%% --*}; args=""; [ "$v" != "$env" ] && args=--${v#* --}
  env $env timeout -k 10 120 python tools/augment_bench.py --no-cpu-baseline --iters 50 $args > gpurun_out/scan.json 2>/dev/null || exit $?
  python -c "import json;d=json.load(open('gpurun_out/scan.json'));print('$v', d['us_per_call'], d['value'], d['roofline']['frac'])"
done
