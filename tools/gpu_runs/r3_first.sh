# Round 3 first GPU pass: GPU tests, smoke, headline bench, bench --gpus 2 spawn rehearsal (gloo, one GPU)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3a
export TMPDIR=/tmp
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3a/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r3a/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3a/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/r3a/smoke.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > gpurun_out/r3a/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(grep '^{' gpurun_out/r3a/bench.log | cut -c1-400)"; [ $rc -eq 0 ] || exit $rc
PAGEVEC_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 3 --warmup 2 --batch 512 --quality-steps 0 --recall 256 > gpurun_out/r3a/spawn2.log 2>&1
rc=$?; echo "spawn2 rc=$rc $(grep '^{' gpurun_out/r3a/spawn2.log | cut -c1-300)"; exit $rc
