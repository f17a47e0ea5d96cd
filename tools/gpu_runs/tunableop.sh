# hipBLASLt solution tuning with PyTorch TunableOp for a bench model: tune once (results CSV
# written under gpurun_out/), then time the bench reading the tuned table vs default.
#   gpurun -- 'bash tools/gpu_runs/tunableop.sh bert'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
M=${1:-bert}
export PYTORCH_TUNABLEOP_FILENAME=$PWD/gpurun_out/tunableop_${M}%d.csv
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_VERBOSE=1 timeout -k 10 900 python -u bench.py --model $M --steps 5 --warmup 3 --quality-steps 0 --recall 0 > gpurun_out/tune_$M.log 2>&1
rc=$?; echo "tune rc=$rc"; tail -1 gpurun_out/tune_$M.log | cut -c1-160; ls -la gpurun_out/tunableop_${M}*.csv
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --model $M --steps 20 --quality-steps 0 --recall 0 > gpurun_out/tuned_off_$r.log 2>&1
  echo "default: $(tail -1 gpurun_out/tuned_off_$r.log | cut -c1-150)"
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=0 timeout -k 10 300 python bench.py --model $M --steps 20 --quality-steps 0 --recall 0 > gpurun_out/tuned_on_$r.log 2>&1
  rc=$?; echo "tuned rc=$rc: $(tail -1 gpurun_out/tuned_on_$r.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
done
