cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof_cdssm2
timeout -k 10 600 python -m pytest tests -m gpu -q -x > gpurun_out/t.log 2>&1; rc=$?; tail -5 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
(cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/prof_cdssm2/cdssm -o cdssm -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --recall 0 --eager-compare 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_cdssm2/cdssm.log 2>&1); rc=$?; echo "cdssm rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --eager-compare 0 > gpurun_out/b.log 2>&1; rc=$?; tail -1 gpurun_out/b.log
