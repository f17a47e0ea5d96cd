cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 500 python tools/quality_run.py --preset cdssm_ngram_bf16 --batch 512 --steps 600 --eval-every 100 > gpurun_out/quality_cdssm.log 2>&1; rc=$?; cat gpurun_out/quality_cdssm.log | grep step; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/quality_run.py --preset mlp_xgpu --batch 1024 --steps 600 --eval-every 200 > gpurun_out/quality_mlp.log 2>&1; rc=$?; cat gpurun_out/quality_mlp.log | grep step
