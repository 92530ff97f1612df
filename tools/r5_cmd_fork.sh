set -o pipefail
T=gpurun_out/r5_fork; mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_netops.py tests/test_abi.py tests/test_decoders.py -m gpu -q --timeout 200 --timeout-method thread > $T/tests.log 2>&1; trc=$?
tail -2 $T/tests.log; grep -E "^(FAILED|ERROR)|GUARD|returncode" $T/tests.log | head
PROF=1 bash tools/r5_ab.sh r5_fork kitti-resnet-san 2 "fork:" "nofork:--no-fork" || exit $?
exit $trc
