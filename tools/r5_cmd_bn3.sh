set -o pipefail
T=gpurun_out/r5_bn3; mkdir -p $T
timeout -k 10 500 python -u -m pytest tests/test_netops.py tests/test_abi.py -m gpu -q --timeout 200 --timeout-method thread -k "not backward_captured" > $T/tests.log 2>&1; rc=$?
tail -3 $T/tests.log; grep -E "^(FAILED|ERROR)" $T/tests.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u bench.py --probe-only --probe-backend nccl > $T/probe_n1.json 2> $T/probe_n1.err; rc=$?
echo "[probe] rc=$rc"; cat $T/probe_n1.json
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --gpus 2 --dist-backend gloo --probe-backend gloo --steps 5 --warmup 3 --no-cpu-baseline --no-kernel-timing > $T/bench_g2_gloo.json 2> $T/bench_g2_gloo.err; rc=$?
echo "[g2 gloo] rc=$rc"; tail -c 400 $T/bench_g2_gloo.json
[ $rc -ne 0 ] && exit $rc
PROF=1 bash tools/r5_ab.sh r5_bn3 kitti-resnet-san 2 "bnres:" "bnres2048:PSFM_BN_RES_MAXM=2048@@" "miopen:--fused-nets bias,gn" || exit $?
timeout -k 10 200 python -u -m pytest tests/test_netops.py -m gpu -q --timeout 150 --timeout-method thread -k "backward_captured" > $T/tests_capture.log 2>&1; rc=$?
tail -3 $T/tests_capture.log; grep -E "GUARD|REFUSED|returncode|assert" $T/tests_capture.log | head
exit $rc
