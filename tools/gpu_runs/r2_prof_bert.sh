# Kernel stats of the BERT step (config 4).
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pbert
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pbert/bert -- python3 bench.py --model bert --steps 8 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/pbert/bert.log 2>&1
echo "bert rc=$?"
