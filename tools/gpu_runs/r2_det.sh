# Deterministic reduction mode: determinism + conv/DDP GPU tests, headline bench default vs --deterministic 1.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/det
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "determin or conv or ddp or direct or cdssm or colsum or adam" > gpurun_out/det/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/det/pytest.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/det/pytest.log | head -20; exit $rc; }
for v in 0 1; do
  timeout -k 10 300 python bench.py --recall 0 --eager-compare 0 --quality-steps 0 --steps 30 --deterministic $v > gpurun_out/det/bench_$v.log 2>&1
  rc=$?; echo "det=$v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/det/bench_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
