# Round 6: reference precision (dtype="fp32") dense layers on the fp32-MFMA GEMM, the explicit
# loss / L2 norm / column sums on their fp32 kernels: tests, then the reference-precision bench
# (the reference's own config: char level, batch 128, fp32) and a kernel profile of it.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_f32
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_conv_f32_gpu.py tests/test_kernels_gpu.py -x -q --timeout 300 --timeout-method thread -k "f32 or fp32 or linear or wgrad or l2norm or explicit or colsum" > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model cdssm_char --dtype fp32 --batch 128 --recall 0 --eager-compare 0 > $O/bench_char_fp32.log 2>&1 || exit $?
tail -1 $O/bench_char_fp32.log | cut -c1-300
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o p -- python3 $GRAFT_REPO_ROOT/bench.py --model cdssm_char --dtype fp32 --batch 128 --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof.log 2>&1 || exit $?
f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/prof_summary.py $f --steps 13 --title "cdssm_char fp32 (reference precision) step kernels, round 6" --cmd "rocprofv3 --kernel-trace --stats -- python3 bench.py --model cdssm_char --dtype fp32 --batch 128 --steps 10 --warmup 3" > $O/stats.md && head -24 $O/stats.md
