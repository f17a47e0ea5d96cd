# PMC passes over the page-tower reduce5 and dW kernels (tools/reduce_ab.py, no reduce6 arms).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bpmc
export TMPDIR=/tmp
run() {  # name counters...
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --kernel-trace --pmc "$@" --output-format csv -d gpurun_out/bpmc/$name -- python3 tools/reduce_ab.py --rb "" --rounds 1 --iters 2 > gpurun_out/bpmc/$name.log 2>&1
  local rc=$?; echo "$name rc=$rc"; return $rc
}
run p1 SQ_WAVES SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY &&
run p2 SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE GRBM_COUNT &&
run p3 TCC_HIT_sum TCC_MISS_sum
