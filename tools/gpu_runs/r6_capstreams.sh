# capture the CDSSM step WITH its side streams; one configuration per call
# (a segfault ends the call).  usage: r6_capstreams.sh <tag> [env assignments...]
cd $GRAFT_REPO_ROOT
tag=$1; shift
O=$GRAFT_REPO_ROOT/gpurun_out/r6_capstreams; mkdir -p $O
env PAGEVEC_CAPTURE_STREAMS=1 AMD_LOG_LEVEL=2 "$@" timeout -k 10 240 python -X faulthandler -u -m pytest tests/test_kernels_gpu.py -k "hipgraph_step_matches_eager and cdssm" -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/$tag.log 2>&1
rc=$?; echo "$tag rc=$rc"; tail -5 $O/$tag.log; exit 0
