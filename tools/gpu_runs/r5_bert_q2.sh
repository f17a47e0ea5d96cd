# BERT recipe variance: two runs per arm of the bench protocol (200 steps) around the new preset.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_bq2
export TMPDIR=/tmp
o=gpurun_out/r5_bq2
B="python -u bench.py --model bert --steps 3 --warmup 3 --eager-compare 0"
for arm in "lr2e-5:" "lr3e-5:--set lr=3e-5" "lr5e-5w20:--set lr=5e-5 --set lr_warmup_steps=20"; do
  name=${arm%%:*}; args=${arm#*:}
  for rep in 1 2; do
    timeout -k 10 200 $B $args > $o/${name}_$rep.log 2>&1
    rc=$?; echo "$name rep $rep rc=$rc $(grep '^{' $o/${name}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["recall_at_10"], d["loss_after_quality_steps"])')"; [ $rc -eq 0 ] || exit $rc
  done
done
