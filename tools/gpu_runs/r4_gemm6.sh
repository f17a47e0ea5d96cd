# Round 4: GEMM v6 (four fat waves, register staging) vs v2 / hipBLASLt; v6 numerics via the engine tests
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_gemm6
export TMPDIR=/tmp
PAGEVEC_GEMM_V6=1 timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "gemm_engine" > gpurun_out/r4_gemm6/pytest.log 2>&1
rc=$?; echo "pytest(v6) rc=$rc $(tail -1 gpurun_out/r4_gemm6/pytest.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_engine_micro.py --rounds 3 > gpurun_out/r4_gemm6/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; grep '^{' gpurun_out/r4_gemm6/micro.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], 'v2', d['engine_tflops'], 'v6', d['engine_v6_tflops'], 'lib', d['library_tflops'], 'err6', '%.1e' % d['v6_max_rel_err'])
"; exit $rc
