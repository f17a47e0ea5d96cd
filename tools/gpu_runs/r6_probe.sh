# Round 6 probes: the W = 8 loss shape on the current kernels (fused glue), and a kernel
# timeline of the MLP (config 3) graph step to place its copyBuffer launches.
cd $GRAFT_REPO_ROOT
O=$GRAFT_REPO_ROOT/gpurun_out/r6_probe
mkdir -p $O
timeout -k 10 300 python tools/ib_micro.py --M 16384,131072 --ib 7 > $O/ib_micro.log 2>&1 || exit $?
cat $O/ib_micro.log | tail -6
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_mlp -o p -- python3 $GRAFT_REPO_ROOT/bench.py --model mlp --steps 10 --warmup 3 --recall 0 --eager-compare 0 --quality-steps 0 > $O/prof_mlp.log 2>&1 || exit $?
t=$(find $O/prof_mlp -name "*kernel_trace.csv" | head -1)
cd $GRAFT_REPO_ROOT && python tools/timeline.py $t > $O/timeline_mlp.txt && grep -c . $O/timeline_mlp.txt && grep -n "copyBuffer" $O/timeline_mlp.txt | head -20
