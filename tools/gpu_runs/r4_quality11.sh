# Round 4: chunked CDSSM preset with embedding dropout 0.125 (nibble mask path): tests, quality, speed
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_quality11
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "conv_pool_fwd_bwd or new_config_training_curve or recall_quality or role_split or word_vocab" > gpurun_out/r4_quality11/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_quality11/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
timeout -k 10 400 python -u bench.py --model chunked_cdssm > gpurun_out/r4_quality11/bench_$i.log 2>&1
rc=$?; echo "bench rc=$rc $(grep '^{' gpurun_out/r4_quality11/bench_$i.log | python3 -c 'import json,sys;d=json.loads(sys.stdin.read());print(d["value"], d["ms_per_step"], d.get("recall_at_10"))')"; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python -u bench.py --quality-steps 0 --recall 0 --eager-compare 0 --steps 30 > gpurun_out/r4_quality11/bench_cdssm.log 2>&1
rc=$?; echo "headline rc=$rc $(grep '^{' gpurun_out/r4_quality11/bench_cdssm.log | cut -c100-175)"; exit $rc
