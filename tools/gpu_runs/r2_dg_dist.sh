# Direct flat-gradient writes under data parallelism: 2-rank gloo tests on one GPU, then
# the multi-rank bench rehearsal.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_distributed_gpu.py tests/test_kernels_gpu.py -k "ddp or direct or cross_gpu" -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_dgdist.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/pytest_dgdist.log
[ $rc -eq 0 ] || exit $rc
bash tools/gpu_runs/dist_rehearsal.sh
