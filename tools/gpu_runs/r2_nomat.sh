# No materialised zero gradients for non-differentiable outputs (argmax, prob, acc): GPU tests + bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/nomat
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/nomat/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/nomat/pytest.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/nomat/pytest.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --recall 0 --eager-compare 0 --quality-steps 0 --steps 40 > gpurun_out/nomat/b_$i.log 2>&1
  rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/nomat/b_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
for M in mlp chunked; do
  timeout -k 10 300 python bench.py --model $M --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/nomat/b_$M.log 2>&1
  rc=$?; echo "$M rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/nomat/b_$M.log)"; [ $rc -eq 0 ] || exit $rc
done
