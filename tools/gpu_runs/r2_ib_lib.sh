# Same-box A/B of the loss kernels (ib_micro at W=1 and W=8 shapes) and the CDSSM bench
# between the current library and lib/variants/$1.so.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$PWD/dnn_page_vectors_amd/lib/variants/$1.so
for r in 1 2; do
  for L in "" $V; do
    tag=${L:+variant}; tag=${tag:-current}
    PAGEVEC_HIP_LIB=$L timeout -k 10 200 python tools/ib_micro.py --M 16384,131072 > gpurun_out/ibl_$tag.log 2>&1 || exit 1
    PAGEVEC_HIP_LIB=$L timeout -k 10 200 python bench.py --steps 30 --warmup 5 --quality-steps 0 --recall 0 --eager-compare 0 > gpurun_out/ibb_$tag.log 2>&1 || exit 1
    echo "$tag r$r $(grep -o 'M=[0-9]*: fwd+bwd [0-9.]* ms' gpurun_out/ibl_$tag.log | tr '\n' ' ') $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ibb_$tag.log)"
  done
done
