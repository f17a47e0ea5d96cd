# Round 4: v7 with the pinned K-step order (sched_barrier per step) at A prefetch depth 1/2/3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_c7sched
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/conv_micro.py --variants 0,17477,17541,17605,16709 --rounds 5 > gpurun_out/r4_c7sched/conv_micro.log 2>&1
rc=$?; grep '^{' gpurun_out/r4_c7sched/conv_micro.log; exit $rc
