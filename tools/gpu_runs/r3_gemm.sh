# Round 3: GEMM engine numerics + micro-benchmark vs hipBLASLt
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3d
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "gemm_engine or mx_fp8" > gpurun_out/r3d/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r3d/pytest.log)"; [ $rc -le 1 ] || exit $rc
[ $rc -eq 0 ] || grep -E "Error|assert|FAILED|Mismatch|Greatest" gpurun_out/r3d/pytest.log | head -20
timeout -k 10 300 python tools/gemm_engine_micro.py > gpurun_out/r3d/gemm_micro.log 2>&1
rc=$?; echo "micro rc=$rc"; grep '^{' gpurun_out/r3d/gemm_micro.log; exit $rc
