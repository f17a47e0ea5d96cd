# Longer retrieval-quality runs (fresh synthetic batches per step, Recall@1/10/100 on 2048
# held-out pairs every 1000 steps): CDSSM headline config and the MLP config, B = 4096.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/qlong
export TMPDIR=/tmp
timeout -k 10 500 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 4096 --steps 6000 --eval-every 1000 > gpurun_out/qlong/cdssm.log 2>&1
rc=$?; echo "cdssm rc=$rc"; grep -v "amdgpu.ids" gpurun_out/qlong/cdssm.log | tail -8; [ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python -u tools/quality_run.py --preset mlp_xgpu --batch 4096 --steps 6000 --eval-every 1000 > gpurun_out/qlong/mlp.log 2>&1
rc=$?; echo "mlp rc=$rc"; grep -v "amdgpu.ids" gpurun_out/qlong/mlp.log | tail -8
