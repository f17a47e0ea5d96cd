# Round 4: v7 timing ablations (max-only epilogue / no A reads / no chunk barriers / all three)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_c7abl
export TMPDIR=/tmp
timeout -k 10 400 python -u tools/conv_micro.py --variants 0,16581,16709,16965,17349 --rounds 5 > gpurun_out/r4_c7abl/conv_micro.log 2>&1
rc=$?; grep '^{' gpurun_out/r4_c7abl/conv_micro.log | grep ms_median; exit $rc
