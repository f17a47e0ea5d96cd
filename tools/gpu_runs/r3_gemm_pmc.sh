# Round 3: PMC pass of the GEMM engine v2 / v3 / hipBLASLt at 8192^3
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3gp
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r3gp/p1 -o p1 --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY -- python3 tools/gemm_engine_micro.py --only square_8192 --iters 2 --rounds 1 > gpurun_out/r3gp/p1.log 2>&1
rc=$?; echo "p1 rc=$rc"; exit $rc
