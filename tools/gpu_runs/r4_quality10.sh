# Round 4: the new longpage_cdssm preset: fp32 parity arm + bench quality
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_quality10
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "new_config_training_curve" > gpurun_out/r4_quality10/parity.log 2>&1
rc=$?; echo "parity rc=$rc $(tail -1 gpurun_out/r4_quality10/parity.log)"; grep "HIP bf16" gpurun_out/r4_quality10/parity.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u bench.py --model chunked_cdssm > gpurun_out/r4_quality10/bench.log 2>&1
rc=$?; echo "bench rc=$rc $(grep '^{' gpurun_out/r4_quality10/bench.log | cut -c1-120) R@10 $(grep '^{' gpurun_out/r4_quality10/bench.log | python3 -c 'import json,sys;print(json.loads(sys.stdin.read()).get("recall_at_10"))')"; exit $rc
