#!/bin/bash
# Backward-chain cache / issue counters of the CDSSM step, streams concurrent (default) vs one stream
set -o pipefail
D=$GRAFT_REPO_ROOT/gpurun_out/r5_bwd_pmc; mkdir -p $D
cd /tmp && export TMPDIR=/tmp
CMD="python3 $GRAFT_REPO_ROOT/bench.py --model cdssm --steps 5 --warmup 2 --recall 0 --quality-steps 0 --eager-compare 0"
PMC="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_WAIT_INST_ANY SQ_LDS_BANK_CONFLICT TCC_HIT_sum TCC_MISS_sum TCP_TOTAL_CACHE_ACCESSES_sum GRBM_GUI_ACTIVE"
timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $D/conc -o conc --pmc $PMC -- $CMD > $D/conc.log 2>&1
rc=$?; echo "concurrent rc=$rc"; [ $rc -eq 0 ] || exit $rc
PAGEVEC_QUERY_STREAM=0 PAGEVEC_EARLY_SORT=0 timeout -s KILL 150 rocprofv3 --kernel-trace --output-format csv -d $D/serial -o serial --pmc $PMC -- $CMD > $D/serial.log 2>&1
rc=$?; echo "serial rc=$rc"; exit $rc
