# rocprofv3 per-kernel stats of the headline bench step.
#   gpurun --timeout 600 -- 'bash tools/gpu_runs/prof_bench.sh [model]'
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/prof
export TMPDIR=/tmp
M=${1:-cdssm}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/$M -- python3 bench.py --model $M --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/prof/$M.log 2>&1
rc=$?; echo "prof rc=$rc"; tail -1 gpurun_out/prof/$M.log
