# the reference's own run configuration end to end (dssm_cnn_v2/cnn_dssm_th.py: char 250 / 5000,
# B 128, J 3, 16000 + 4000 samples per epoch, 5 epochs, Adam, fp32) on synthetic pairs
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r4_refrun && mkdir -p gpurun_out/r4_refrun
START=$(date +%s.%N)
timeout -k 10 600 python -u -m dnn_page_vectors_amd train --preset reference_char --synthetic --set experiment_root_directory=$GRAFT_REPO_ROOT/gpurun_out/r4_refrun/exp > gpurun_out/r4_refrun/train.log 2>&1
rc=$?
END=$(date +%s.%N)
echo "rc=$rc wall_s=$(python3 -c "print(round($END-$START,1))")" | tee gpurun_out/r4_refrun/wall.txt
tail -3 gpurun_out/r4_refrun/train.log
find gpurun_out/r4_refrun/exp -name "*.safetensors" -delete
exit $rc
