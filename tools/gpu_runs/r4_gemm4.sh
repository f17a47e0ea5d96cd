# Round 4: the 8-phase GEMM (v4) vs v2 / v3 / hipBLASLt at the model shapes; early dTable sort A/B
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_gemm4
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/gemm_engine_micro.py --rounds 3 > gpurun_out/r4_gemm4/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; grep '^{' gpurun_out/r4_gemm4/micro.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], 'v2', d['engine_tflops'], 'v4', d['engine_v4_tflops'], 'v3', d.get('engine_v3_tflops'), 'lib', d['library_tflops'], 'err4', '%.1e' % d['v4_max_rel_err'])
"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "emitted_keys or word_vocab or dtable or training_curve_hip_matches_torch or hipgraph" > gpurun_out/r4_gemm4/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_gemm4/pytest.log)"; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for es in 0 1; do
PAGEVEC_EARLY_SORT=$es timeout -k 10 300 python -u bench.py --quality-steps 0 --recall 0 --eager-compare 0 --steps 30 > gpurun_out/r4_gemm4/bench_es${es}_$i.log 2>&1
rc=$?; echo "early_sort=$es rc=$rc $(grep '^{' gpurun_out/r4_gemm4/bench_es${es}_$i.log | cut -c1-200)"; [ $rc -eq 0 ] || exit $rc
done; done
