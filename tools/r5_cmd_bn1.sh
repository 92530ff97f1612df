set -o pipefail
mkdir -p gpurun_out/r5_bn1
timeout -k 10 400 python -u -m pytest tests/test_netops.py tests/test_pack3d.py tests/test_abi.py -m gpu -q --timeout 200 --timeout-method thread -k "netops or forms or dw_matrix or abi" > gpurun_out/r5_bn1/netops_tests.log 2>&1; rc=$?
tail -3 gpurun_out/r5_bn1/netops_tests.log; grep -E "^(FAILED|ERROR)" gpurun_out/r5_bn1/netops_tests.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --probe-only --probe-backend nccl > gpurun_out/r5_bn1/probe_n1.json 2> gpurun_out/r5_bn1/probe_n1.err; rc=$?
echo "[probe] rc=$rc"; cat gpurun_out/r5_bn1/probe_n1.json; grep "comm probe" gpurun_out/r5_bn1/probe_n1.err
[ $rc -ne 0 ] && exit $rc
PROF=1 bash tools/r5_ab.sh r5_bn1 kitti-resnet-san 2 "bnres:" "miopen:--fused-nets bias,gn"
