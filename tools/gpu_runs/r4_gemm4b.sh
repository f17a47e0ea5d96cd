# Round 4: GEMM v4 with the grouped tile order vs v2 / hipBLASLt
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_gemm4b
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/gemm_engine_micro.py --rounds 3 > gpurun_out/r4_gemm4b/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; grep '^{' gpurun_out/r4_gemm4b/micro.log | python3 -c "
import sys, json
for l in sys.stdin:
    d = json.loads(l); print(d['shape'], 'v2', d['engine_tflops'], 'v4', d['engine_v4_tflops'], 'v4g0', d['engine_v4_group0_tflops'], 'v3', d.get('engine_v3_tflops'), 'lib', d['library_tflops'], 'err4', '%.1e' % d['v4_max_rel_err'])
"; exit $rc
