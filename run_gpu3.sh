cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for m in mlp bert chunked; do
  timeout -k 10 300 python bench.py --model $m --steps 10 --warmup 3 --recall 0 > gpurun_out/bench_$m.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/bench_$m.log; exit 1; }
  tail -1 gpurun_out/bench_$m.log
done
timeout -k 10 600 python bench.py --backend torch --batch 512 --steps 5 --warmup 2 --recall 0 > gpurun_out/bench_eager.log 2>&1; echo "eager rc=$?"; tail -1 gpurun_out/bench_eager.log
timeout -k 10 300 python bench.py --batch 512 --steps 10 --warmup 3 --recall 0 > gpurun_out/bench_hip512.log 2>&1; tail -1 gpurun_out/bench_hip512.log
