# Retrieval quality on the GPU box: CDSSM (config 2) and MLP (config 3), eager steps,
# fresh synthetic batches per step, Recall@1/10/100 on held-out pages every 250 steps.
#   gpurun --timeout 900 -- 'bash tools/gpu_runs/quality.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 4096 --steps 1500 --eval-every 250 > gpurun_out/quality_cdssm.log 2>&1
rc=$?; echo "cdssm rc=$rc"; grep -v "amdgpu.ids" gpurun_out/quality_cdssm.log | tail -7
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quality_run.py --preset mlp_xgpu --batch 4096 --steps 1500 --eval-every 250 > gpurun_out/quality_mlp.log 2>&1
rc=$?; echo "mlp rc=$rc"; grep -v "amdgpu.ids" gpurun_out/quality_mlp.log | tail -7
