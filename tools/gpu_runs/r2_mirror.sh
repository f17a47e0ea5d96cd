# bf16 mirrors written by the Adam kernel: GPU tests, then same-box A/B on MLP / chunked / BERT.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py \
  -k "mirror or adam or hipgraph or train_step or direct" > gpurun_out/mirror_tests.log 2>&1
rc=$?; tail -3 gpurun_out/mirror_tests.log; [ $rc -eq 0 ] || exit $rc
M=mlp ENVB="PAGEVEC_NO_MIRROR=1" bash tools/gpu_runs/r2_ab_model.sh || exit 1
M=chunked ENVB="PAGEVEC_NO_MIRROR=1" bash tools/gpu_runs/r2_ab_model.sh || exit 1
M=bert S=10 ENVB="PAGEVEC_NO_MIRROR=1" bash tools/gpu_runs/r2_ab_model.sh
