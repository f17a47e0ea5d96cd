cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench_default.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -1 gpurun_out/bench_default.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --model mlp > gpurun_out/bench_mlp.log 2>&1
rc=$?; echo "bench mlp rc=$rc"; tail -1 gpurun_out/bench_mlp.log
