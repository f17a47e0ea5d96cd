# BERT recipe robustness (bench protocol: 200 quality steps, Recall@10 on 2048 held-out pairs).
# usage: r5_bert_q3.sh "<name>:<bench args>" ... (each arm run REPS times)
cd $GRAFT_REPO_ROOT
o=gpurun_out/r5_bq3; mkdir -p $o
export TMPDIR=/tmp
REPS=${REPS:-3}
B="python -u bench.py --model bert --steps 3 --warmup 3 --eager-compare 0"
for arm in "$@"; do
  name=${arm%%:*}; args=${arm#*:}
  for rep in $(seq 1 $REPS); do
    timeout -k 10 200 $B $args > $o/${name}_$rep.log 2>&1
    rc=$?; echo "$name rep $rep rc=$rc $(grep '^{' $o/${name}_$rep.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["recall_at_10"], d["loss_after_quality_steps"])')"; [ $rc -eq 0 ] || exit $rc
  done
done
