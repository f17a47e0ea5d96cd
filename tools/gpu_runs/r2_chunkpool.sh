# Fused chunk mean-pool: its test + chunked GPU tests + chunked bench x3.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cpool
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "chunk or longpage or big_model or fp8" > gpurun_out/cpool/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/cpool/pytest.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/cpool/pytest.log | head; exit $rc; }
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --model chunked --recall 0 --eager-compare 0 --steps 50 > gpurun_out/cpool/b_$i.log 2>&1
  rc=$?; echo "chunked rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/cpool/b_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
