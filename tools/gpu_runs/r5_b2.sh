# BERT preset change (softmax scale 20, no clip) + attention QG defaults: the GPU tests that
# use the preset / attention, the bench with the new defaults, two more recipe arms.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_b2
export TMPDIR=/tmp
o=gpurun_out/r5_b2
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py -k "bert or attention or new_config_training_curve" -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > $o/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 $o/pytest.log)"; [ $rc -eq 0 ] || { tail -60 $o/pytest.log; exit $rc; }
B="python -u bench.py --model bert --steps 10 --warmup 5 --eager-compare 0"
timeout -k 10 240 $B > $o/bert_default.log 2>&1
rc=$?; echo "bert default rc=$rc $(tail -1 $o/bert_default.log | cut -c1-300)"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 $B --set inbatch_gamma=40 > $o/bert_g40.log 2>&1
rc=$?; echo "bert g40 rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 $B --set inbatch_gamma=30 > $o/bert_g30.log 2>&1
rc=$?; echo "bert g30 rc=$rc"; [ $rc -eq 0 ] || exit $rc
