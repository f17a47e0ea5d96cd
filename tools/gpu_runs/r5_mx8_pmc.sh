# MX fp8 GEMM: timing at config 5's shapes, then two PMC passes (counters in their own runs).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_mx8
export TMPDIR=/tmp
o=gpurun_out/r5_mx8
timeout -k 10 120 python -u tools/mx8_micro.py > $o/micro.log 2>&1
rc=$?; echo "micro rc=$rc $(tail -1 $o/micro.log)"; [ $rc -eq 0 ] || exit $rc
CMD="python3 tools/mx8_micro.py --iters 3"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $o/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > $o/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $o/p2 -o p2 --pmc SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES -- $CMD > $o/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; [ $rc -eq 0 ] || exit $rc
python3 tools/pmc_summary.py $o/p1 $o/p2 --match gemm_mx8 > $o/summary.md
cat $o/summary.md
