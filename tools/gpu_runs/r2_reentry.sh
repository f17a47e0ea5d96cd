# Re-entry check after a container rebuild: GPU tests, smoke, headline bench.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/reentry
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/reentry/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/reentry/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/reentry/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/reentry/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py > gpurun_out/reentry/bench_cdssm.log 2>&1
rc=$?; echo "cdssm rc=$rc $(tail -1 gpurun_out/reentry/bench_cdssm.log | cut -c1-200)"
