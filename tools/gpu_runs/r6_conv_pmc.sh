# Round 6: conv forward v7 vs its no-A-read ablation under PMC (two counter passes) — where do
# the MFMA waves lose the 28 % of the matrix pipe?
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r6_conv_pmc; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
CMD="python3 $GRAFT_REPO_ROOT/tools/conv_micro.py --variants 0,16709 --rounds 1 --iters 2"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $D/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE -- $CMD > $D/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $D/p2 -o p2 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD -- $CMD > $D/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py $D/p1 $D/p2 --match conv_pool_fwd7 > $D/pmc.md && cat $D/pmc.md
