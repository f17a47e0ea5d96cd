# Round 3: what the embedding dropout (mask hashing in conv fwd staging, dW, dTable reduce) costs per step
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3dc
for arm in element none element none; do
  timeout -k 10 200 python bench.py --model cdssm --steps 30 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 --set embed_dropout_mode=$arm > gpurun_out/r3dc/b_$arm.log 2>&1
  rc=$?; echo "dropout=$arm rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/r3dc/b_$arm.log)"; [ $rc -eq 0 ] || exit $rc
done
