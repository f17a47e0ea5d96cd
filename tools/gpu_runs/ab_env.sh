# A/B of an environment switch on the headline bench, interleaved (A B A B), after the
# conv + graph GPU tests.   gpurun -- 'bash tools/gpu_runs/ab_env.sh VAR valA valB'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
VAR=$1; A=$2; B=$3; MODEL=${4:-cdssm}; TESTS=${5:-conv or hipgraph}
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "$TESTS" > gpurun_out/pytest_ab.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/pytest_ab.log
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python bench.py --model $MODEL --steps 30 --warmup 5 --quality-steps 0 --recall 0 --eager-compare 0 > gpurun_out/ab_${v}_$r.log 2>&1
    rc=$?; echo "$VAR=$v run $r rc=$rc $(tail -1 gpurun_out/ab_${v}_$r.log | python -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
    [ $rc -eq 0 ] || exit $rc
  done
done
