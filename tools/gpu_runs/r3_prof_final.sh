# Round 3 (second session): kernel stats of the headline step and the MLP step with the new defaults
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pf
export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf/cdssm -o cdssm -- python3 bench.py --model cdssm --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/pf/cdssm.log 2>&1
rc=$?; echo "cdssm rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pf/mlp -o mlp -- python3 bench.py --model mlp --steps 20 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/pf/mlp.log 2>&1
rc=$?; echo "mlp rc=$rc"; exit $rc
