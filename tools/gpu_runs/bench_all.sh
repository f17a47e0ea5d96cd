# All BASELINE configs on one GPU (headline cdssm + mlp / bert / chunked) and a rocprofv3 kernel profile of cdssm.
#   gpurun --timeout 1200 -- 'bash tools/gpu_runs/bench_all.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
for M in cdssm mlp bert chunked; do
  timeout -k 10 300 python bench.py --model $M > gpurun_out/bench_$M.log 2>&1
  rc=$?; echo "$M rc=$rc"; tail -1 gpurun_out/bench_$M.log
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/cdssm -- python3 bench.py --model cdssm --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/prof/cdssm.log 2>&1
echo "prof rc=$?"
