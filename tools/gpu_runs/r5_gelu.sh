# bias + GELU vector kernels v1 / v2: numerics (both) and the micro.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_gelu
export TMPDIR=/tmp
o=gpurun_out/r5_gelu
timeout -k 10 200 python -u -m pytest "tests/test_kernels_gpu.py::test_add_layernorm_and_bias_gelu" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $o/pytest.log)"; [ $rc -eq 0 ] || { tail -40 $o/pytest.log; exit $rc; }
timeout -k 10 200 python -u tools/gelu_micro.py > $o/gelu_micro.log 2>&1
rc=$?; echo "gelu micro rc=$rc $(tail -1 $o/gelu_micro.log)"; [ $rc -eq 0 ] || exit $rc
