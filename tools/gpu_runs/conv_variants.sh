# A/B of conv forward schedule variants (one process, interleaved) + bit-exactness checks.
#   gpurun --timeout 600 -- 'bash tools/gpu_runs/conv_variants.sh 0,261,265,269'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python tools/conv_micro.py --variants ${1:-0} --rounds 5 > gpurun_out/conv_variants.log 2>&1
rc=$?; echo "micro rc=$rc"; grep -v amdgpu.ids gpurun_out/conv_variants.log
