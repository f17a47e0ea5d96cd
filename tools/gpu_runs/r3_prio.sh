# Round 3: headline step with the eager step on a high-priority stream (side streams normal)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3pr
python3 -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
for arm in 0 1 0 1; do
  PAGEVEC_SIDE_PRIORITY=$arm timeout -k 10 200 python bench.py --model cdssm --steps 30 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r3pr/b$arm.log 2>&1
  rc=$?; echo "prio=$arm rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3pr/b$arm.log)"; [ $rc -eq 0 ] || exit $rc
done
