# reduce8 diagnosis: uniform vs Zipf ids (same-address LDS atomics on hot rows?)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r8
export TMPDIR=/tmp
timeout -k 10 200 python3 tools/table_chain_ab.py --uniform --seg 4096 --rounds 3 > gpurun_out/r8/chain_uniform.log 2>&1
rc=$?; cat gpurun_out/r8/chain_uniform.log; exit $rc
