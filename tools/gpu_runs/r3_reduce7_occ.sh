# Round 3: dTable reduce7 at 8 waves/SIMD (64 VGPRs) vs 6 (74), plus PMC of reduce7 at the bench shape
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r7
export TMPDIR=/tmp
CMD="python3 tools/reduce_ab.py --rb= --rounds 3"
timeout -k 10 300 python3 tools/reduce_ab.py --rb= --rounds 7 > gpurun_out/r7/ab.log 2>&1
rc=$?; grep '^{' gpurun_out/r7/ab.log; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r7/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VMEM_RD SQ_WAIT_INST_LDS SQ_INSTS_VALU GRBM_GUI_ACTIVE -- $CMD > gpurun_out/r7/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r7/p2 -o p2 --pmc TCC_HIT_sum TCC_MISS_sum SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVES SQ_LDS_BANK_CONFLICT GRBM_COUNT -- $CMD > gpurun_out/r7/p2.log 2>&1
rc=$?; echo "p2 rc=$rc"; exit $rc
