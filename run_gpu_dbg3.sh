cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 200 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 200 --eval-every 100 --print-each > gpurun_out/dbg3.log 2>&1
rc=$?; echo "rc=$rc"; grep -v "amdgpu.ids\|^frame" gpurun_out/dbg3.log | grep -v launched | tail -30; grep launched gpurun_out/dbg3.log | tail -2
