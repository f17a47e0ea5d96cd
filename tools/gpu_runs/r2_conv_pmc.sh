# Round 2: PMC counters of the production conv forward (v3), one pass per counter group
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc
export TMPDIR=/tmp
CMD="python3 tools/conv_micro.py --variants 0 --rounds 1 --iters 2"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > gpurun_out/pmc/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/pmc/p2 -o p2 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_INST_LEVEL_LDS SQ_LDS_IDX_ACTIVE GRBM_COUNT -- $CMD > gpurun_out/pmc/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; exit $rc
