# Round 4: quality -- recall guard value, parity arms for the new configs, chunked-CDSSM recipe sweep
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_quality
export TMPDIR=/tmp
timeout -k 10 500 python -u -m pytest tests/test_kernels_gpu.py -x -v -s --timeout 400 --timeout-method thread -p no:cacheprovider -k "recall_quality_guard or new_config_training_curve" > gpurun_out/r4_quality/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r4_quality/tests.log)"; grep -E "recall@10|HIP bf16|FAILED|Error" gpurun_out/r4_quality/tests.log | head; [ $rc -eq 0 ] || exit $rc
i=0
for S in "" "lr=3e-3" "inbatch_gamma=60" "lr=3e-3 inbatch_gamma=60" "dropout_prob=[0.0,0.5]" "lr=3e-3 dropout_prob=[0.0,0.5]"; do
  i=$((i+1)); ARGS=""; for kv in $S; do ARGS="$ARGS --set $kv"; done
  timeout -k 10 300 python -u bench.py --model chunked_cdssm --steps 10 --warmup 3 --eager-compare 0 $ARGS > gpurun_out/r4_quality/cc_$i.log 2>&1
  rc=$?; echo "[$S] rc=$rc $(tail -1 gpurun_out/r4_quality/cc_$i.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("recall_at_10"), d.get("final_loss", d.get("loss")))' 2>&1 | tail -1)"; [ $rc -eq 0 ] || exit $rc
done
