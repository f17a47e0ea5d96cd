# Headline preset with the in-batch softmax scale 40: GPU tests (incl. the Recall@10 guard), headline bench x2.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gfin
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/gfin/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/gfin/pytest.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/gfin/pytest.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 400 python bench.py > gpurun_out/gfin/b_$i.log 2>&1
  rc=$?; echo "bench rc=$rc $(tail -1 gpurun_out/gfin/b_$i.log | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"recall_at_10": [0-9.]*\|"final_loss": [-0-9.a-zA-Z]*' | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
