# dW kernel: compile-time dropout mode vs runtime mode (two processes each, interleaved), conv GPU tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/dwdm
export TMPDIR=/tmp
for i in 1 2; do
  for m in runtime tmpl; do
    PAGEVEC_DW_DM=$m timeout -k 10 200 python tools/reduce_ab.py --rb "" --rounds 3 > gpurun_out/dwdm/ab_${m}_$i.log 2>&1
    rc=$?; echo "$m rc=$rc $(tail -1 gpurun_out/dwdm/ab_${m}_$i.log)"; [ $rc -eq 0 ] || exit $rc
  done
done
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv or cdssm or determin or ddp" > gpurun_out/dwdm/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/dwdm/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --recall 0 --eager-compare 0 --quality-steps 0 --steps 40 > gpurun_out/dwdm/b_$i.log 2>&1
  rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/dwdm/b_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
