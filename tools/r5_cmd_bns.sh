set -o pipefail
T=gpurun_out/r5_bns; mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_netops.py tests/test_abi.py -m gpu -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1; rc=$?
tail -2 $T/tests.log; grep -E "^(FAILED|ERROR)" $T/tests.log | head
[ $rc -ne 0 ] && exit $rc
PROF=1 bash tools/r5_ab.sh r5_bns kitti-resnet-san 3 "bnall:--fused-nets bias,gn,bnall" "bnres:"
