# every preset through `train --synthetic` for 2 short epochs (+ encode for two): finite losses,
# every epoch with batches
cd $GRAFT_REPO_ROOT
rm -rf gpurun_out/r5_presets && mkdir -p gpurun_out/r5_presets
for P in reference_char reference_v1 cdssm_ngram_bf16 mlp_xgpu bert_dp8 longpage_fp8 longpage_cdssm lstm tiny_dssm_cpu; do
  timeout -k 10 240 python -u -m dnn_page_vectors_amd train --preset $P --synthetic --set experiment_root_directory=/tmp/pv_$P --set nb_epoch=2 --set num_validation_samples=2048 > gpurun_out/r5_presets/$P.log 2>&1
  rc=$?
  echo "$P rc=$rc $(tail -1 gpurun_out/r5_presets/$P.log | cut -c1-330)"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
