# BERT (config 4) quality: full-depth fp32 parity arm, then a recipe sweep in the bench protocol
# (200 optimizer steps, Recall@10 on 2048 held-out pairs) over lr / warmup / softmax scale / clip.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_bert
export TMPDIR=/tmp
out=gpurun_out/r5_bert
run() {  # name, timeout, command...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$n.log 2>&1
  local rc=$?
  echo "$n rc=$rc $(tail -1 $out/$n.log | cut -c1-600)"
  case $rc in 0) ;; *) exit $rc ;; esac
}
B="python -u bench.py --model bert --steps 3 --warmup 3 --eager-compare 0"
if [ "$1" = "a" ]; then
run parity12 400 python -u tools/bert_parity.py --layers 12 --batch 64 --steps 200
run base 200 $B
run lr1e4_w50 200 $B --set lr=1e-4 --set lr_warmup_steps=50
run lr1e4_w50_noclip_g20 200 $B --set lr=1e-4 --set lr_warmup_steps=50 --set cos_clip=False --set inbatch_gamma=20
else
run lr3e5_w20 200 $B --set lr=3e-5 --set lr_warmup_steps=20
run lr5e5_w50 200 $B --set lr=5e-5 --set lr_warmup_steps=50
run lr2e5_noclip_g20 200 $B --set cos_clip=False --set inbatch_gamma=20
run lr2e5_g20 200 $B --set inbatch_gamma=20
fi
