# attention.hip QG (16-row groups per wave) variants: numerics for every QG, then the micro.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_attn
export TMPDIR=/tmp
o=gpurun_out/r5_attn
timeout -k 10 300 python -u -m pytest "tests/test_kernels_gpu.py::test_fused_attention_packed_qkv" "tests/test_kernels_gpu.py::test_packed_attention_qkv_projection_grads" "tests/test_kernels_gpu.py::test_masked_attention" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $o/pytest.log)"; [ $rc -eq 0 ] || { tail -40 $o/pytest.log; exit $rc; }
timeout -k 10 200 python -u tools/attn_micro.py > $o/attn_micro.log 2>&1
rc=$?; echo "attn micro rc=$rc $(tail -1 $o/attn_micro.log)"; [ $rc -eq 0 ] || exit $rc
