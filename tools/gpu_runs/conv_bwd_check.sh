# conv backward numerics tests + backward micro-benchmark (Zipf ids)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_kernels_gpu.py -x -q -m gpu -k "conv or dtable or cdssm" --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_conv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bwd_micro.py --ids zipf --epw 0,512 > gpurun_out/bwd_micro_zipf.log 2>&1
rc=$?; echo "zipf rc=$rc"; grep -v amdgpu.ids gpurun_out/bwd_micro_zipf.log
