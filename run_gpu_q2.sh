cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 4096 --steps 1500 --eval-every 250 --graph 0 > gpurun_out/q2_lr1e-3.log 2>&1
rc=$?; echo "lr1e-3 rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/q2_lr1e-3.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 4096 --steps 1500 --eval-every 250 --graph 0 --lr 0.004 > gpurun_out/q2_lr4e-3.log 2>&1
rc=$?; echo "lr4e-3 rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/q2_lr4e-3.log | tail -8
[ $rc -eq 0 ] || exit $rc
TORCH_BLAS_PREFER_HIPBLASLT=0 timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 200 --eval-every 100 --graph 1 --print-each > gpurun_out/q2_graph_rocblas.log 2>&1
rc=$?; echo "graph rocblas rc=$rc"; grep -v "amdgpu.ids\|^frame\|launched" gpurun_out/q2_graph_rocblas.log | tail -5; grep launched gpurun_out/q2_graph_rocblas.log | tail -1
