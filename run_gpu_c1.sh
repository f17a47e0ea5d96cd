cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/conv_micro.py --variants 0,257,258,259,0 --rounds 5 > gpurun_out/conv_c1.log 2>&1
rc=$?; echo "micro rc=$rc"; cat gpurun_out/conv_c1.log | grep -v amdgpu.ids
