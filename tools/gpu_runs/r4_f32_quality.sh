# reference char config at its batch of 128: fp32 native vs bf16, 500 steps + Recall@10
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_f32q
for DT in fp32 bf16; do
timeout -k 10 300 python -u bench.py --model cdssm_char --dtype $DT --batch 128 --steps 20 --warmup 5 > gpurun_out/r4_f32q/char_$DT.log 2>&1
rc=$?; echo "$DT rc=$rc"; grep '^{' gpurun_out/r4_f32q/char_$DT.log | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"], d["dtype"], d.get("final_loss"), d.get("quality_loss"), d.get("recall_at_10"))'; [ $rc -eq 0 ] || exit $rc
done
