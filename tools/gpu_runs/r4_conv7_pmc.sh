# Round 4: PMC of conv forward v7 (production) vs v4, plus the dropout-off timing ablation
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_c7pmc
export TMPDIR=/tmp
timeout -k 10 300 python -u tools/conv_micro.py --variants 4096,0 --rounds 5 --p 0 > gpurun_out/r4_c7pmc/conv_micro_p0.log 2>&1
rc=$?; grep '^{' gpurun_out/r4_c7pmc/conv_micro_p0.log; [ $rc -eq 0 ] || exit $rc
CMD="python3 tools/conv_micro.py --variants 4096,0 --rounds 1 --iters 3"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_c7pmc/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > gpurun_out/r4_c7pmc/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r4_c7pmc/p2 -o p2 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES -- $CMD > gpurun_out/r4_c7pmc/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py gpurun_out/r4_c7pmc/p1 gpurun_out/r4_c7pmc/p2 --match conv_pool_fwd > gpurun_out/r4_c7pmc/summary.md
cat gpurun_out/r4_c7pmc/summary.md
