# Same-box A/B of an environment switch on one model's bench.
#   gpurun -- 'M=bert S=10 ENVB="PAGEVEC_COLSUM=0" bash tools/gpu_runs/r2_ab_model.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
B="python bench.py --model ${M:-cdssm} --steps ${S:-30} --warmup 5 --eager-compare 0 --quality-steps 0 --recall 0"
for r in 1 2; do
  timeout -k 10 200 $B > gpurun_out/abm_a$r.log 2>&1 || exit 1
  timeout -k 10 200 env $ENVB $B > gpurun_out/abm_b$r.log 2>&1 || exit 1
  echo "A $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abm_a$r.log)  B[$ENVB] $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abm_b$r.log)"
done
