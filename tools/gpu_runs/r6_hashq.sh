# Quality A/B of the dropout group hash: the round-6 mix24 stream (default library) vs the
# round-5 mix32 stream (variant build PV_DROP_HASH_LEGACY), headline bench protocol (20 timed
# steps, 1000-step quality phase, Recall@10 on 2048 held-out pairs), four training seeds each.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_hashq
mkdir -p $O
LEG=$GRAFT_REPO_ROOT/dnn_page_vectors_amd/lib/variants/libpagevec_hip_PV_DROP_HASH_LEGACY_1.so
for s in 1337 11 22 33; do
  for arm in new legacy; do
    if [ $arm = legacy ]; then export PAGEVEC_HIP_LIB=$LEG; else unset PAGEVEC_HIP_LIB; fi
    timeout -k 10 300 python bench.py --eager-compare 0 --set seed=$s > $O/${arm}_$s.log 2>&1 || exit $?
    echo "$arm seed $s $(tail -1 $O/${arm}_$s.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'], d['recall_at_10'], d['loss_after_quality_steps'])")"
  done
done
