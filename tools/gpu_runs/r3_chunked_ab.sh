# Round 3: chunked (config 5) bench with the MX fp8 page bag vs the bf16 counts GEMM, + kernel profiles
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ch
export TMPDIR=/tmp
for arm in 1 0 1; do
  PAGEVEC_FP8_BAG=$arm timeout -k 10 300 python bench.py --model chunked > gpurun_out/r3ch/bench_fp8bag$arm.log 2>&1
  rc=$?; echo "fp8bag=$arm rc=$rc $(grep '^{' gpurun_out/r3ch/bench_fp8bag$arm.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d.get("recall_at_10"))')"
  [ $rc -eq 0 ] || exit $rc
done
for M in chunked cdssm; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r3ch/prof_$M -- python3 bench.py --model $M --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r3ch/prof_$M.log 2>&1
  rc=$?; echo "prof $M rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
