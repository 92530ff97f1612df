set -o pipefail
T=gpurun_out/r5_netin; mkdir -p $T
timeout -k 10 300 python -u -m pytest tests/test_netops.py tests/test_abi.py -m gpu -q -k "net_input or pose_input or posenet or stem or abi" --timeout 120 --timeout-method thread > $T/tests.log 2>&1; rc=$?
tail -2 $T/tests.log; grep -E "^(FAILED|ERROR)" $T/tests.log | head
[ $rc -ne 0 ] && exit $rc
PROF=1 bash tools/r5_ab.sh r5_netin kitti-resnet-san 3 "netin:" "nonetin:--no-net-inputs"
