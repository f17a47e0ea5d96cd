# Round 4: forward-emitted dTable keys -- tests + headline A/B (PAGEVEC_FWD_EMIT=0/1)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_emit
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "conv_pool or emitted or word_vocab or role_split or dtable or hipgraph" > gpurun_out/r4_emit/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r4_emit/tests.log)"; grep -E "FAILED|Error" gpurun_out/r4_emit/tests.log | head; [ $rc -eq 0 ] || exit $rc
for i in 1 2; do
for E in 0 1; do
PAGEVEC_FWD_EMIT=$E timeout -k 10 300 python -u bench.py --steps 30 --warmup 5 --recall 0 --eager-compare 0 --quality-steps 0 > gpurun_out/r4_emit/bench_$E.$i.log 2>&1
rc=$?; echo "emit=$E rc=$rc $(tail -1 gpurun_out/r4_emit/bench_$E.$i.log | cut -c1-150)"; [ $rc -eq 0 ] || exit $rc
done; done
