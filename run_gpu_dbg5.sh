cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 100 --eval-every 100 --graph 0 --print-each > gpurun_out/dbg5a.log 2>&1
rc=$?; echo "eager nosync rc=$rc"; grep -v "amdgpu.ids\|^frame\|launched" gpurun_out/dbg5a.log | tail -8; grep launched gpurun_out/dbg5a.log | tail -1
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 100 --eval-every 100 --graph 1 --pool 100 --print-each > gpurun_out/dbg5b.log 2>&1
rc=$?; echo "graph pooled rc=$rc"; grep -v "amdgpu.ids\|^frame\|launched" gpurun_out/dbg5b.log | tail -8; grep launched gpurun_out/dbg5b.log | tail -1
