cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 12 --eval-every 6 --graph 1 --sync-each > gpurun_out/dbg2_graph_sync.log 2>&1
rc=$?; echo "release graph sync rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/dbg2_graph_sync.log | tail -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 12 --eval-every 6 --graph 1 --print-each > gpurun_out/dbg2_graph_nosync.log 2>&1
rc=$?; echo "release graph nosync rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/dbg2_graph_nosync.log | tail -20
