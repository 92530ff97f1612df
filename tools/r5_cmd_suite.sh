set -o pipefail
bash tools/r4_suite.sh r5_suite_final || exit $?
# the default bench line (as the driver runs it) on the stamped profiles: roofline traffic + rocprof time + cpu_baseline
mkdir -p gpurun_out/r5_default
timeout -k 10 500 python -u bench.py > gpurun_out/r5_default/bench_default.json 2> gpurun_out/r5_default/bench_default.err; rc=$?
cat gpurun_out/r5_default/bench_default.json; exit $rc
