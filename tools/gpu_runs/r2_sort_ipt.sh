# Radix sort tile size A/B (items per thread 4 / 16 / 32) at the conv-backward shapes.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/sipt
export TMPDIR=/tmp
timeout -k 10 200 python tools/sort_micro.py --iters 30 > gpurun_out/sipt/ab.log 2>&1
rc=$?; tail -3 gpurun_out/sipt/ab.log; exit $rc
