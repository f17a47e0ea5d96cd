cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_f32
timeout -k 10 300 python -u bench.py --model cdssm_char --dtype fp32 --batch 128 --steps 20 --warmup 3 --quality-steps 0 --recall 0 > gpurun_out/r4_f32/bench_native.log 2>&1
rc=$?; echo "native rc=$rc"; grep '^{' gpurun_out/r4_f32/bench_native.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
bash tools/gpu_runs/r4_refrun.sh
