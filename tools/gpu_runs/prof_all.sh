# rocprofv3 kernel stats for every bench config (one short run each).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_all
export TMPDIR=/tmp
for M in cdssm mlp bert chunked cdssm_char; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_all/$M -- python3 bench.py --model $M --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/prof_all/$M.log 2>&1
  rc=$?; echo "$M rc=$rc $(tail -1 gpurun_out/prof_all/$M.log | cut -c1-160)"
  [ $rc -eq 0 ] || exit $rc
done
