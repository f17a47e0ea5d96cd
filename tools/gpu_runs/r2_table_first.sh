# Table-gradient-first conv backward + own DDP bucket for embedding tables: GPU tests of
# the conv / DDP / trainer paths, then the headline bench (W = 1 must not regress).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/tfirst
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "conv or ddp or direct or trainer or hipgraph or cdssm or distributed" > gpurun_out/tfirst/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/tfirst/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
  timeout -k 10 300 python bench.py --recall 0 --eager-compare 0 --quality-steps 0 --steps 40 > gpurun_out/tfirst/bench_$i.log 2>&1
  rc=$?; echo "cdssm rc=$rc $(tail -1 gpurun_out/tfirst/bench_$i.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
done
