# chunked quality-phase diagnosis: graph vs eager, fp8 vs bf16
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3ch
for g in 0 1; do
  timeout -k 10 200 python bench.py --model chunked --graph $g --steps 10 --warmup 5 > gpurun_out/r3ch/dbg_graph$g.log 2>&1
  rc=$?; echo "graph=$g rc=$rc"; grep "quality step" gpurun_out/r3ch/dbg_graph$g.log; grep -o '"recall_at_10": [0-9.]*' gpurun_out/r3ch/dbg_graph$g.log; [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 200 python bench.py --model mlp --steps 10 --warmup 5 --quality-steps 300 > gpurun_out/r3ch/dbg_mlp.log 2>&1
rc=$?; echo "mlp rc=$rc"; grep "quality step" gpurun_out/r3ch/dbg_mlp.log; grep -o '"recall_at_10": [0-9.]*' gpurun_out/r3ch/dbg_mlp.log; exit $rc
