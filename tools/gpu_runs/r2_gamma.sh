# In-batch / cross-GPU softmax temperature for the CDSSM headline: Recall@10 vs GAMMA (2000 steps each).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/gamma
export TMPDIR=/tmp
for g in ${GAMMAS:-10 20 40}; do
  timeout -k 10 300 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 4096 --steps 2000 --eval-every 1000 --no-initial-eval --set GAMMA=$g > gpurun_out/gamma/g$g.log 2>&1
  rc=$?; echo "gamma=$g rc=$rc $(grep recall gpurun_out/gamma/g$g.log | tail -1)"; [ $rc -eq 0 ] || exit $rc
done
