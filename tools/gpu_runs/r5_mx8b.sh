# MX fp8 GEMM staging buffers 2 vs 3: numerics (bit-identical + fp32 reference), micro, chunked A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_mx8
export TMPDIR=/tmp
o=gpurun_out/r5_mx8
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -k "gemm_mx8 or fp8 or mx_fp8" tests/test_bag_gemm_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $o/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 $o/tests.log)"; [ $rc -eq 0 ] || { tail -30 $o/tests.log; exit $rc; }
timeout -k 10 200 python -u tools/mx8_micro.py > $o/micro_ns.log 2>&1
rc=$?; echo "micro rc=$rc $(tail -1 $o/micro_ns.log)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/step_flag_ab.py --setter pv_gemm_mx8_set_stages --vals 2,3 --preset longpage_fp8 > $o/chunked_ns_ab.txt 2>&1
rc=$?; echo "chunked ab rc=$rc $(tail -1 $o/chunked_ns_ab.txt)"; [ $rc -eq 0 ] || exit $rc
