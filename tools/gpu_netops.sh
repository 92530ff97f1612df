set -u
OUT=gpurun_out; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_netops.py -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/netops_tests.log 2>&1; rc=$?
echo "[netops tests] rc=$rc"; tail -3 $OUT/netops_tests.log
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline --fused-nets > $OUT/bench_fused.json 2> $OUT/bench_fused.err; rc=$?
echo "[bench fused] rc=$rc"; cat $OUT/bench_fused.json | head -c 400; echo
[ $rc -ne 0 ] && exit $rc
timeout -k 10 400 python bench.py --steps 50 --warmup 10 --no-cpu-baseline > $OUT/bench_plain.json 2> $OUT/bench_plain.err; rc=$?
echo "[bench plain] rc=$rc"; cat $OUT/bench_plain.json | head -c 400; echo
[ $rc -ne 0 ] && exit $rc
rm -rf $OUT/prof
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-kernel-timing --fused-nets) > $OUT/prof.log 2>&1; rc=$?
echo "[prof] rc=$rc"
[ $rc -ne 0 ] && exit $rc
python3 tools/summarize_trace.py $OUT/prof/run_kernel_trace.csv $OUT/prof/step_summary.txt; rm -f $OUT/prof/run_kernel_trace.csv
head -40 $OUT/prof/step_summary.txt
