cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 120 python -m pytest tests/test_kernels_gpu.py -q -m gpu -k "conv" -p no:cacheprovider > gpurun_out/pytest_conv.log 2>&1
rc=$?; echo "pytest conv rc=$rc"; tail -2 gpurun_out/pytest_conv.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/quality_run.py --preset cdssm_ngram_bf16 --batch 1024 --steps 800 --eval-every 100 > gpurun_out/quality_cdssm.log 2>&1
rc=$?; echo "q cdssm rc=$rc"; grep -v amdgpu.ids gpurun_out/quality_cdssm.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u tools/quality_run.py --preset mlp_xgpu --batch 1024 --steps 800 --eval-every 200 > gpurun_out/quality_mlp.log 2>&1
rc=$?; echo "q mlp rc=$rc"; grep -v amdgpu.ids gpurun_out/quality_mlp.log | tail -6
