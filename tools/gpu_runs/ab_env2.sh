# Same-box A/B of an environment switch on the headline bench (timing only: no quality phase).
#   gpurun -- 'ENVB="PAGEVEC_DW_STREAM=1" bash tools/gpu_runs/ab_env2.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for r in 1 2; do
  timeout -k 10 150 python bench.py --steps 30 --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0 > gpurun_out/ab_a$r.log 2>&1 || exit 1
  timeout -k 10 150 env $ENVB python bench.py --steps 30 --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0 > gpurun_out/ab_b$r.log 2>&1 || exit 1
  echo "A $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_a$r.log)  B[$ENVB] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_b$r.log)"
done
