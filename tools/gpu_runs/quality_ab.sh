# Recall@10 after the 1000-step quality phase: current library vs a variant (same box).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
V=$PWD/dnn_page_vectors_amd/lib/variants/$1.so
for L in "" $V; do
  PAGEVEC_HIP_LIB=$L timeout -k 10 300 python bench.py --steps 5 --warmup 3 --eager-compare 0 > gpurun_out/qab.log 2>&1
  rc=$?; echo "${L:-current} rc=$rc $(grep -o '"recall_at_10": [0-9.]*\|"loss_after_quality_steps": [0-9.]*' gpurun_out/qab.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
