# One-kernel bag-mean backward prologue: bag / MLP / chunked GPU tests, MLP + chunked benches.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bagbwd
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "bag or mlp or chunk or longpage or big_model or determin or ddp or direct or colsum" > gpurun_out/bagbwd/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/bagbwd/pytest.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/bagbwd/pytest.log | head; exit $rc; }
for M in mlp chunked mlp chunked; do
  timeout -k 10 300 python bench.py --model $M --recall 0 --eager-compare 0 --quality-steps 0 --steps 50 > gpurun_out/bagbwd/b_$M.log 2>&1
  rc=$?; echo "$M rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/bagbwd/b_$M.log)"; [ $rc -eq 0 ] || exit $rc
done
