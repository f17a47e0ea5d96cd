# Round 3: ib3 loss kernels (512-thread WGs, LDS-DMA ring) vs ib2: numerics tests, A/B timing,
# kernel trace at the W = 8 shape
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/ib3
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "inbatch or explicit" > gpurun_out/ib3/tests.log 2>&1
rc=$?; tail -5 gpurun_out/ib3/tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 tools/ib_micro.py --M 16384,131072 --iters 10 --ib 5,3,2,5,3 > gpurun_out/ib3/time.log 2>&1
rc=$?; cat gpurun_out/ib3/time.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/ib3/kt -o kt -- python3 tools/ib_micro.py --M 131072 --iters 3 --ib 5 > gpurun_out/ib3/kt.log 2>&1
rc=$?; echo "kt rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ib3/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- python3 tools/ib_micro.py --M 131072 --iters 3 --ib 5 > gpurun_out/ib3/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; exit $rc
