# Round 3: staggered 4-phase bf16 GEMM (gemm3_kernel) numerics + micro-benchmark vs hipBLASLt
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3g3
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -v --timeout 120 --timeout-method thread -k "gemm_engine" > gpurun_out/r3g3/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/r3g3/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/gemm_engine_micro.py --rounds 3 > gpurun_out/r3g3/micro.log 2>&1
rc=$?; echo "micro rc=$rc"; grep "{" gpurun_out/r3g3/micro.log | python3 -c '
import json,sys
for l in sys.stdin:
    d=json.loads(l); print(d["shape"], "v2", d["engine_tflops"], "v3", d.get("engine_v3_tflops"), "lib", d["library_tflops"], "err3", d.get("v3_max_rel_err"))'
exit $rc
