cd $GRAFT_REPO_ROOT
timeout -k 10 400 python bench.py --no-cpu-baseline > gpurun_out/bench_resident.json 2> gpurun_out/bench_resident.err || exit $?
head -c 300 gpurun_out/bench_resident.json; echo
timeout -k 10 400 python bench.py --no-cpu-baseline --data-path gpu-augment > gpurun_out/bench_gpuaug.json 2> gpurun_out/bench_gpuaug.err || exit $?
head -c 300 gpurun_out/bench_gpuaug.json; echo
