cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export PAGEVEC_DEBUG_KERNELS=1
timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 12 --eval-every 6 --graph 0 --sync-each > gpurun_out/dbg_eager.log 2>&1
rc=$?; echo "eager rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/dbg_eager.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 12 --eval-every 6 --graph 1 --sync-each > gpurun_out/dbg_graph.log 2>&1
rc=$?; echo "graph rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/dbg_graph.log | tail -20
