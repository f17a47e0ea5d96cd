# Round 4: chunked CDSSM recipe confirmation (tanh head, no cosine clip, embedding dropout 0.1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_quality9
export TMPDIR=/tmp
summ() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("recall_at_10"), d.get("loss_after_quality_steps"))'; }
i=0
for S in "lr=3e-3" "lr=3e-3" "lr=3e-3 hidden_dims=300" "lr=2.5e-3"; do
  i=$((i+1)); ARGS="--set cdssm_act=tanh --set cos_clip=False --set dropout_prob=[0.1,0.5]"; for kv in $S; do ARGS="$ARGS --set $kv"; done
  timeout -k 10 400 python -u bench.py --model chunked_cdssm --steps 10 --warmup 3 --eager-compare 0 $ARGS > gpurun_out/r4_quality9/cc_$i.log 2>&1
  rc=$?; echo "chunked_cdssm tanh/noclip/drop0.1 [$S] rc=$rc $(tail -1 gpurun_out/r4_quality9/cc_$i.log | summ 2>&1 | tail -1)"
done
