# bag GEMM lt micro, attention (QG + forward DMA) numerics + micro, BERT-preset GPU tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_misc
export TMPDIR=/tmp
o=gpurun_out/r5_misc
timeout -k 10 200 python -u tools/bag_lt_micro.py > $o/bag_lt_micro.log 2>&1
rc=$?; echo "bag lt micro rc=$rc $(tail -1 $o/bag_lt_micro.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest "tests/test_kernels_gpu.py::test_fused_attention_packed_qkv" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/attn_tests.log 2>&1
rc=$?; echo "attn tests rc=$rc $(tail -1 $o/attn_tests.log)"; [ $rc -eq 0 ] || { tail -30 $o/attn_tests.log; exit $rc; }
timeout -k 10 200 python -u tools/attn_micro.py > $o/attn_micro.log 2>&1
rc=$?; echo "attn micro rc=$rc $(tail -1 $o/attn_micro.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -k "bert or new_config" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $o/bert_tests.log 2>&1
rc=$?; echo "bert tests rc=$rc $(tail -1 $o/bert_tests.log)"; [ $rc -eq 0 ] || { tail -30 $o/bert_tests.log; exit $rc; }
