cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
PAGEVEC_DEBUG_KERNELS=1 timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 100 --eval-every 100 --sync-each > gpurun_out/dbg4a.log 2>&1
rc=$?; echo "debug sync rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/dbg4a.log | grep -v '"debug": {}' | tail -12; grep step gpurun_out/dbg4a.log | tail -2
[ $rc -eq 0 ] || exit $rc
grep -q '"debug": {"' gpurun_out/dbg4a.log && exit 0
timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 100 --eval-every 100 --sync-each > gpurun_out/dbg4b.log 2>&1
rc=$?; echo "release sync rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/dbg4b.log | tail -12
