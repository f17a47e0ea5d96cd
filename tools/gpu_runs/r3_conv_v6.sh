# Round 3: conv forward v6 (three waves per SIMD, 768-thread workgroups) vs v4 (two per SIMD)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/v6
export TMPDIR=/tmp
timeout -k 10 400 python tools/conv_micro.py --variants 0,8204,8236,8268,8220,8252 --rounds 7 > gpurun_out/v6/conv_micro.log 2>&1
rc=$?; grep '^{' gpurun_out/v6/conv_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_micro.py --N 4096 --L 5000 --variants 0,8204,8236 --rounds 5 > gpurun_out/v6/conv_micro_l5000.log 2>&1
rc=$?; grep '^{' gpurun_out/v6/conv_micro_l5000.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_micro.py --N 4096 --L 45 --variants 0,8204,8236 --rounds 5 > gpurun_out/v6/conv_micro_q.log 2>&1
rc=$?; grep '^{' gpurun_out/v6/conv_micro_q.log; exit $rc
