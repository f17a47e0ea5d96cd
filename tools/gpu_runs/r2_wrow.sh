# One-launch backward weight rows: conv GPU tests + headline bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/wrow
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv or dtable or cdssm or determin or weight_rows" > gpurun_out/wrow/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/wrow/pytest.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/wrow/pytest.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py --recall 0 --eager-compare 0 --quality-steps 0 --steps 40 > gpurun_out/wrow/b_$i.log 2>&1
  rc=$?; echo "bench rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/wrow/b_$i.log)"; [ $rc -eq 0 ] || exit $rc
done
