# Round 2: per-kernel profile of the radix sort vs rocPRIM; eager vs graph learning curve
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_sort -o sort -- python3 tools/sort_micro.py --iters 10 > gpurun_out/prof_sort.log 2>&1
rc=$?; echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 240 python -u tools/quality_run.py --graph 0 --batch 512 --steps 300 --eval-every 100 \
   --no-initial-eval > gpurun_out/eager_probe.log 2>&1
rc=$?; echo "eager rc=$rc"; grep -v amdgpu.ids gpurun_out/eager_probe.log | grep preset
exit $rc
