# fp32 (reference-precision) conv tower: numerics tests, then bench native vs all-PyTorch fp32
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_f32
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_conv_f32_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_f32/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_f32/pytest.log)"; grep -E "FAILED|Error|assert" gpurun_out/r4_f32/pytest.log | head -30; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --model cdssm_char --dtype fp32 --batch 128 --steps 10 --warmup 3 --quality-steps 0 --recall 0 > gpurun_out/r4_f32/bench_native.log 2>&1
rc=$?; echo "native rc=$rc"; grep '^{' gpurun_out/r4_f32/bench_native.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
PAGEVEC_F32_NATIVE=0 timeout -k 10 400 python -u bench.py --model cdssm_char --dtype fp32 --batch 128 --steps 5 --warmup 2 --quality-steps 0 --recall 0 > gpurun_out/r4_f32/bench_torch.log 2>&1
rc=$?; echo "torch rc=$rc"; grep '^{' gpurun_out/r4_f32/bench_torch.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
cd /tmp && timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/r4_f32/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --model cdssm_char --dtype fp32 --batch 128 --steps 5 --warmup 2 --quality-steps 0 --recall 0 > $GRAFT_REPO_ROOT/gpurun_out/r4_f32/prof.log 2>&1
echo "prof rc=$?"
