set -o pipefail
T=gpurun_out/r5_invdepth; mkdir -p $T
timeout -k 10 400 python -u -m pytest tests/test_networks.py -m gpu -q --timeout 300 --timeout-method thread > $T/tests.log 2>&1; rc=$?
tail -2 $T/tests.log; grep -E "^(FAILED|ERROR)" $T/tests.log | head
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python -u bench.py --config kitti-packnet-san --steps 20 --warmup 5 --no-cpu-baseline > $T/bench_kitti-packnet-san.json 2> $T/bench.err; rc=$?
cat $T/bench_kitti-packnet-san.json; exit $rc
