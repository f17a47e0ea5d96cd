# Round 4: chunked CDSSM with a tanh Dense head (chunk vectors of both signs before the mean) / no cosine clip
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_quality6
export TMPDIR=/tmp
summ() { python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d.get("recall_at_10"), d.get("loss_after_quality_steps"))'; }
i=0
for S in "cdssm_act=tanh cos_clip=False" "cdssm_act=tanh cos_clip=False lr=1e-3" "cdssm_act=tanh cos_clip=False lr=5e-3" "cdssm_act=tanh" "cos_clip=False"; do
  i=$((i+1)); ARGS=""; for kv in $S; do ARGS="$ARGS --set $kv"; done
  timeout -k 10 400 python -u bench.py --model chunked_cdssm --steps 10 --warmup 3 --eager-compare 0 $ARGS > gpurun_out/r4_quality6/cc_$i.log 2>&1
  rc=$?; echo "chunked_cdssm [$S] rc=$rc $(tail -1 gpurun_out/r4_quality6/cc_$i.log | summ 2>&1 | tail -1)"; [ $rc -eq 0 ] || exit $rc
done
