cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PAGEVEC_DEBUG_KERNELS=1 timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 100 --eval-every 20 --graph 1 > gpurun_out/dbg6.log 2>&1
rc=$?; echo "debug graph nosync rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/dbg6.log | tail -12
