# Fill-free fp8 amax + quantisation: fp8 / chunked GPU tests, chunked bench A/B against the previous commit's numbers.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/fp8q
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "fp8 or chunk or longpage or big_model" > gpurun_out/fp8q/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/fp8q/pytest.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/fp8q/pytest.log | head; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model chunked --recall 0 --eager-compare 0 --steps 50 > gpurun_out/fp8q/b_$i.log 2>&1
  rc=$?; echo "chunked rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/fp8q/b_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
