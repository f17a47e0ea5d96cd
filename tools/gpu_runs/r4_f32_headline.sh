# the headline config (ngram, B 4096, Ld 2000, J 3, cross-GPU loss) at the reference's fp32: native vs all-PyTorch
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_f32h
timeout -k 10 300 python -u bench.py --model cdssm --dtype fp32 --steps 5 --warmup 2 --quality-steps 0 --recall 0 --eager-compare 0 > gpurun_out/r4_f32h/native.log 2>&1
rc=$?; echo "native rc=$rc"; grep '^{' gpurun_out/r4_f32h/native.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
PAGEVEC_F32_NATIVE=0 timeout -k 10 400 python -u bench.py --model cdssm --dtype fp32 --steps 2 --warmup 1 --quality-steps 0 --recall 0 --eager-compare 0 > gpurun_out/r4_f32h/torch.log 2>&1
rc=$?; echo "torch rc=$rc"; grep '^{' gpurun_out/r4_f32h/torch.log | cut -c1-200; tail -3 gpurun_out/r4_f32h/torch.log; exit $rc
