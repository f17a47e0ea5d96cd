# End-of-round check: GPU tests, smoke, every bench config, CDSSM kernel profile.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/final
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/final/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/final/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/final/smoke.log)"; [ $rc -eq 0 ] || exit $rc
for M in cdssm mlp bert chunked cdssm_char; do
  timeout -k 10 400 python bench.py --model $M > gpurun_out/final/bench_$M.log 2>&1
  rc=$?; echo "$M rc=$rc $(tail -1 gpurun_out/final/bench_$M.log | cut -c1-170)"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final/prof_cdssm -- python3 bench.py --model cdssm --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/final/prof_cdssm.log 2>&1
echo "prof rc=$?"
