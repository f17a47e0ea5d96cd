# Kernel stats of the chunked (config 5) and MLP (config 3) steps.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/psmall
export TMPDIR=/tmp
for M in chunked mlp; do
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/psmall/$M -- python3 bench.py --model $M --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/psmall/$M.log 2>&1
  rc=$?; echo "$M rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
