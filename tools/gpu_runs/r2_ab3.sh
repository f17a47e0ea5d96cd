# Same-box three-way A/B of an environment variable's values on one model's bench.
#   gpurun -- 'M=bert S=10 VAR=PAGEVEC_GELU_UNROLL VALS="1 2 4" bash tools/gpu_runs/r2_ab3.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --model ${M:-cdssm} --steps ${S:-30} --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0"
for r in 1 2; do
  line=""
  for v in $VALS; do
    timeout -k 10 200 env $VAR=$v $B > gpurun_out/ab3_$v.log 2>&1 || exit 1
    line="$line $VAR=$v $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab3_$v.log | cut -d' ' -f2)"
  done
  echo "$line"
done
