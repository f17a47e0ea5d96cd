# Distributed step under hipGraph capture (world-1 RCCL group, every collective forced on),
# the RCCL eager rehearsal, and the headline stream-placement A/B.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_dg
export TMPDIR=/tmp
timeout -k 10 420 python -u -m pytest tests/test_rccl_gpu.py tests/test_sparse_rows_gpu.py tests/test_optim_warmup.py -x -v -s --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/r5_dg/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r5_dg/pytest.log)"; grep -E "^(mlp|cdssm) \{" gpurun_out/r5_dg/pytest.log; [ $rc -eq 0 ] || { tail -50 gpurun_out/r5_dg/pytest.log; exit $rc; }
timeout -k 10 300 python tools/step_flag_ab.py --env PAGEVEC_QUERY_STREAM --vals 0,1 > gpurun_out/r5_dg/qstream_ab.txt 2>&1
rc=$?; echo "qstream ab rc=$rc $(tail -1 gpurun_out/r5_dg/qstream_ab.txt)"
