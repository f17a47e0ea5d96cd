# lt_gemm / fp8 bag backward / wide-loss flash kernel tests, the FFN / linear micro, step A/Bs.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_lt
export TMPDIR=/tmp
o=gpurun_out/r5_lt
timeout -k 10 500 python -u -m pytest tests/test_ffn_lt_gpu.py tests/test_bag_gemm_gpu.py "tests/test_kernels_gpu.py::test_inbatch_loss_wide_rows_path" tests/test_distributed_gpu.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $o/pytest.log)"; [ $rc -eq 0 ] || { tail -60 $o/pytest.log; exit $rc; }
timeout -k 10 300 python -u tools/ffn_micro.py > $o/ffn_micro.log 2>&1
rc=$?; echo "ffn micro rc=$rc $(tail -1 $o/ffn_micro.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.transformer --flag LINEAR_LT --preset bert_dp8 --rounds 4 --steps 8 > $o/bert_linear_lt_ab.txt 2>&1
rc=$?; echo "bert linear lt ab rc=$rc $(tail -1 $o/bert_linear_lt_ab.txt)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.loss --flag IB_WIDE --preset bert_dp8 --rounds 4 --steps 8 > $o/bert_ib_wide_ab.txt 2>&1
rc=$?; echo "bert ib wide ab rc=$rc $(tail -1 $o/bert_ib_wide_ab.txt)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_flag_ab.py --module dnn_page_vectors_amd.ops.embedding --flag FP8_BWD --preset longpage_fp8 > $o/chunked_fp8bwd_ab.txt 2>&1
rc=$?; echo "chunked fp8 bwd ab rc=$rc $(tail -1 $o/chunked_fp8bwd_ab.txt)"; [ $rc -eq 0 ] || exit $rc
