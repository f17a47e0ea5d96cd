# Same-box A/B of the current kernel library against dnn_page_vectors_amd/lib/variants/<name>.so:
# conv fwd + backward micro-benchmarks and the headline bench, interleaved A B A B.
#   gpurun -- 'bash tools/gpu_runs/lib_ab.sh libpagevec_hip_prev'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$PWD/dnn_page_vectors_amd/lib/variants/$1.so
: > gpurun_out/lib_ab.log
for r in 1 2; do
  for L in "" $V; do
    tag=${L:+variant}; tag=${tag:-current}
    echo "== $tag run $r" >> gpurun_out/lib_ab.log
    PAGEVEC_HIP_LIB=$L timeout -k 10 200 python tools/bwd_micro.py --epw 512 --rounds 2 >> gpurun_out/lib_ab.log 2>&1 &&
    PAGEVEC_HIP_LIB=$L timeout -k 10 200 python tools/conv_micro.py --variants 0 --rounds 2 >> gpurun_out/lib_ab.log 2>&1 &&
    PAGEVEC_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 30 --quality-steps 0 --recall 0 --eager-compare 0 >> gpurun_out/lib_ab.log 2>&1
    rc=$?; echo "$tag run $r rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
grep -E "^==|\"emit\"|fwd_ms|pairs/s" gpurun_out/lib_ab.log | sed -e 's/"data".*//' | cut -c1-220
