# encode() (serving) throughput for each model.   gpurun -- 'bash tools/gpu_runs/encode.sh'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
: > gpurun_out/encode_bench.log
for M in cdssm mlp cdssm_char bert; do
  timeout -k 10 200 python tools/encode_bench.py --model $M >> gpurun_out/encode_bench.log 2>&1
  rc=$?; echo "$M rc=$rc"; tail -1 gpurun_out/encode_bench.log
  [ $rc -eq 0 ] || exit $rc
done
