# Round 3 (end): bench line for every model config on the final tree
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/allm
export TMPDIR=/tmp
for m in mlp bert chunked_cdssm cdssm_char; do
  timeout -k 10 400 python3 bench.py --model $m > gpurun_out/allm/$m.log 2>&1
  rc=$?; echo "$m rc=$rc $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"recall_at_10": [0-9.]*' gpurun_out/allm/$m.log | tr '\n' ' ')"; [ $rc -eq 0 ] || exit $rc
done
