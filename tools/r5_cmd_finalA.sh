set -o pipefail
T=gpurun_out/r5_finalA_tests; mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_netops.py tests/test_abi.py -m gpu -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1; rc=$?
tail -2 $T/tests.log; grep -E "^(FAILED|ERROR)" $T/tests.log | head
[ $rc -ne 0 ] && exit $rc
bash tools/r5_final.sh r5_finalA kitti-resnet-san kitti-packnet-san
