cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_qbwd -o q -- python3 tools/qbwd_micro.py --shapes 4096x45 --rounds 2 > gpurun_out/prof_qbwd.log 2>&1
rc=$?; echo "prof rc=$rc"; exit $rc
