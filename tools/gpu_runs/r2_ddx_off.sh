# Dense-dX off by default: conv / DDP / determinism / trainer GPU tests, headline bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ddx2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv or dtable or cdssm or determin or ddp or direct or trainer or hipgraph or dense_dx" > gpurun_out/ddx2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/ddx2/pytest.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error" gpurun_out/ddx2/pytest.log | head; exit $rc; }
for i in 1 2; do
  timeout -k 10 300 python bench.py > gpurun_out/ddx2/b_$i.log 2>&1
  rc=$?; echo "bench rc=$rc $(tail -1 gpurun_out/ddx2/b_$i.log | cut -c1-220)"; [ $rc -eq 0 ] || exit $rc
done
