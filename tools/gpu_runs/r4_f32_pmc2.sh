cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_f32_pmc2
export TMPDIR=/tmp
CMD="python3 tools/f32_micro.py --iters 3"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_f32_pmc2/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > gpurun_out/r4_f32_pmc2/p1.log 2>&1
echo "p1 rc=$?"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_f32_pmc2/p2 -o p2 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES -- $CMD > gpurun_out/r4_f32_pmc2/p2.log 2>&1
echo "p2 rc=$?"
