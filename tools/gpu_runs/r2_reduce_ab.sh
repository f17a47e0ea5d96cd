# reduce5 vs reduce6 (weight-row gathers of RB rounds in flight), same process.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/rab
export TMPDIR=/tmp
timeout -k 10 200 python tools/reduce_ab.py > gpurun_out/rab/ab.log 2>&1
rc=$?; cat gpurun_out/rab/ab.log | tail -8; exit $rc
