# Round 3: localise the ib3 disagreement (tools/ib_diag.py) on the shapes of test_inbatch_loss_split_shapes
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ib3
export TMPDIR=/tmp
timeout -k 10 240 python3 tools/ib_diag.py --B 4096 --M 16384 --clip 0 > gpurun_out/ib3/diag.log 2>&1
rc=$?; cat gpurun_out/ib3/diag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 tools/ib_diag.py --B 700 --M 5000 --clip 1 >> gpurun_out/ib3/diag.log 2>&1
rc=$?; tail -12 gpurun_out/ib3/diag.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python3 tools/ib_diag.py --B 4096 --M 16384 --clip 1 >> gpurun_out/ib3/diag.log 2>&1
rc=$?; tail -12 gpurun_out/ib3/diag.log; exit $rc
