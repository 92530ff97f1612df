# A/B of netops variants: rocprofv3 kernel trace of tools/netops_bench.py per library build
set -u
OUT=$GRAFT_REPO_ROOT/gpurun_out/nab; rm -rf $OUT; mkdir -p $OUT; export TMPDIR=/tmp
run() {  # name, args...
  local name=$1; shift
  (cd /tmp && timeout -k 10 180 rocprofv3 --kernel-trace --output-format csv -d $OUT/$name -o run -- python3 $GRAFT_REPO_ROOT/tools/netops_bench.py "$@") > $OUT/$name.log 2>&1; local rc=$?
  echo "[$name] rc=$rc"; [ $rc -ne 0 ] && { tail -5 $OUT/$name.log; exit $rc; }
  grep -E "^(fused|ref) " $OUT/$name.log
  python3 $GRAFT_REPO_ROOT/tools/summarize_grid.py $(ls $OUT/$name/run_kernel_trace.csv 2>/dev/null || find $OUT/$name -name '*kernel_trace.csv' | head -1) "k_bn_,k_gn_,MIOpenBatchNorm,Rowwise,ComputeInternal,GroupNorm,threshold,clamp,elementwise" > $OUT/$name.txt
  grep -E 'k_bn_|k_gn_|MIOpenBatch' $OUT/$name.txt
}
run ref --mode ref
run base
for v in notree gs64 t128 t128gs128 t64u8gs64; do run $v --lib $GRAFT_REPO_ROOT/build/variants/$v.so; done
