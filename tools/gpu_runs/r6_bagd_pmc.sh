# Round 6: bagd_mm_kernel (dense-count bag GEMMs) vs the library's GEMMs under PMC (two counter
# passes over tools/bag_gemm_micro.py): MFMA busy, waits, LDS.
cd $GRAFT_REPO_ROOT
D=$GRAFT_REPO_ROOT/gpurun_out/r6_bagd_pmc; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
CMD="python3 $GRAFT_REPO_ROOT/tools/bag_gemm_micro.py"
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $D/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_COEXEC_CYCLES GRBM_GUI_ACTIVE -- $CMD > $D/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d $D/p2 -o p2 --pmc SQ_INSTS_LDS SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES SQ_INSTS_VMEM_RD -- $CMD > $D/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
cd $GRAFT_REPO_ROOT && python tools/pmc_summary.py $D/p1 $D/p2 --match bagd_mm,Cijk > $D/pmc.md && cat $D/pmc.md
