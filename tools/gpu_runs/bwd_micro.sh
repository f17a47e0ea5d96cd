cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python tools/bwd_micro.py --ids zipf > gpurun_out/bwd_micro_zipf.log 2>&1
rc=$?; echo "zipf rc=$rc"; grep -v amdgpu.ids gpurun_out/bwd_micro_zipf.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python tools/bwd_micro.py --ids uniform > gpurun_out/bwd_micro_uniform.log 2>&1
rc=$?; echo "uniform rc=$rc"; grep -v amdgpu.ids gpurun_out/bwd_micro_uniform.log
