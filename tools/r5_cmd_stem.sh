set -o pipefail
T=gpurun_out/r5_stem; mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_netops.py -m gpu -q -k "stem or add_relu or forked or bn_act" --timeout 120 --timeout-method thread > $T/tests.log 2>&1; rc=$?
tail -2 $T/tests.log; grep -E "^(FAILED|ERROR)" $T/tests.log | head
[ $rc -ne 0 ] && exit $rc
PROF=1 bash tools/r5_ab.sh r5_stem kitti-resnet-san 3 "stem:" "nostem:--no-stem-pool"
