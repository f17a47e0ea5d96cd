# Round 3: conv forward late-wave epilogue deferral (OPT 16 / spread 48, +/- setprio) A/B vs production
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/stag
export TMPDIR=/tmp
timeout -k 10 400 python tools/conv_micro.py --variants 0,4125,4157,4124,4108 --rounds 7 > gpurun_out/stag/conv_micro.log 2>&1
rc=$?; grep '^{' gpurun_out/stag/conv_micro.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python tools/conv_micro.py --N 4096 --L 5000 --variants 0,4125,4157 --rounds 5 > gpurun_out/stag/conv_micro_l5000.log 2>&1
rc=$?; grep '^{' gpurun_out/stag/conv_micro_l5000.log; exit $rc
