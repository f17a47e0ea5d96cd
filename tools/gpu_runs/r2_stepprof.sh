# Round 2: per-kernel stats of the headline CDSSM step (13 dispatched steps) + bench line
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
MODEL=${MODEL:-cdssm}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_step_$MODEL -o step -- python3 bench.py --model $MODEL --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/prof_step_$MODEL.log 2>&1
rc=$?; echo "prof rc=$rc"; grep -v amdgpu.ids gpurun_out/prof_step_$MODEL.log | tail -2
exit $rc
