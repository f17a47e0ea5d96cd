# Round 4: chunked CDSSM recipes (chunk pooling of the conv features, lr, softmax scale)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_quality5
export TMPDIR=/tmp
summ() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("recall_at_10"), d.get("loss_after_quality_steps"))'; }
i=0
for S in "chunk_pool=mean_features" "chunk_pool=mean_features lr=5e-3" "chunk_pool=mean_features inbatch_gamma=20" "chunk_pool=max lr=5e-3" "lr=3e-3 dropout_prob=[0.1,0.5]"; do
  i=$((i+1)); ARGS=""; for kv in $S; do ARGS="$ARGS --set $kv"; done
  timeout -k 10 400 python -u bench.py --model chunked_cdssm --steps 10 --warmup 3 --eager-compare 0 $ARGS > gpurun_out/r4_quality5/cc_$i.log 2>&1
  rc=$?; echo "chunked_cdssm [$S] rc=$rc $(tail -1 gpurun_out/r4_quality5/cc_$i.log | summ 2>&1 | tail -1)"; [ $rc -eq 0 ] || exit $rc
done
