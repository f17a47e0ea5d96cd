# Round 3: glue removal (strided l2norm backward gradient, conv bias pointers): tests, bench, kernel trace
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/glue
export TMPDIR=/tmp
timeout -k 10 900 python3 -u -m pytest -x -q --timeout 400 --timeout-method thread tests/test_kernels_gpu.py tests/test_distributed_gpu.py \
  -k "l2norm or inbatch or cross_gpu or cdssm or train or mlp or bert or chunk" > gpurun_out/glue/tests.log 2>&1
rc=$?; tail -3 gpurun_out/glue/tests.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 40 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/glue/b$r.log 2>&1
  rc=$?; echo "bench $r: $(tail -1 gpurun_out/glue/b$r.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
done
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/glue/cdssm -o cdssm -- python3 bench.py --model cdssm --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/glue/prof.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
