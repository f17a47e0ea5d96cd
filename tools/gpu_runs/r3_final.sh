# Round 3 (third session): full GPU test suite, smoke, headline + chunked bench, headline kernel stats
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3h
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -s --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r3h/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r3h/pytest.log)"; [ $rc -le 1 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3h/smoke.log 2>&1
rc2=$?; echo "smoke rc=$rc2 $(tail -1 gpurun_out/r3h/smoke.log)"; [ $rc2 -eq 0 ] || exit $rc2
timeout -k 10 300 python bench.py > gpurun_out/r3h/bench_headline.log 2>&1
rc3=$?; echo "headline rc=$rc3 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"recall_at_10": [0-9.]*' gpurun_out/r3h/bench_headline.log | tr '\n' ' ')"; [ $rc3 -eq 0 ] || exit $rc3
timeout -k 10 300 python bench.py --model chunked > gpurun_out/r3h/bench_chunked.log 2>&1
rc4=$?; echo "chunked rc=$rc4 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"recall_at_10": [0-9.]*' gpurun_out/r3h/bench_chunked.log | tr '\n' ' ')"; [ $rc4 -eq 0 ] || exit $rc4
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3h/cdssm -o cdssm -- python3 bench.py --model cdssm --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r3h/cdssm_prof.log 2>&1
rc5=$?; echo "prof rc=$rc5"; [ $rc5 -eq 0 ] || exit $rc5
exit $rc
