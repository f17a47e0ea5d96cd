# Round 4: wide-vector (D = 768) cross-GPU loss without reduce-scatter -- multi-rank GPU tests,
# and a forced-collective (RCCL world 1) BERT step under a kernel trace: no ReduceScatter kernel
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_wide
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_distributed_gpu.py -x -v --timeout 250 --timeout-method thread -p no:cacheprovider > gpurun_out/r4_wide/tests.log 2>&1
rc=$?; echo "tests rc=$rc $(tail -1 gpurun_out/r4_wide/tests.log)"; grep -E "FAILED|Error" gpurun_out/r4_wide/tests.log | head; [ $rc -eq 0 ] || exit $rc
PAGEVEC_FORCE_DIST=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=29533 timeout -s KILL 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r4_wide/bert -o bert -- python3 bench.py --model bert --steps 4 --warmup 2 --recall 0 --eager-compare 0 --quality-steps 0 --graph 0 > gpurun_out/r4_wide/bert.log 2>&1
rc=$?; echo "bert rc=$rc $(tail -1 gpurun_out/r4_wide/bert.log | cut -c1-160)"; [ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import csv
rows = list(csv.DictReader(open("gpurun_out/r4_wide/bert/bert_kernel_stats.csv")))
rccl = [(r["Name"][:90], r["Calls"]) for r in rows if "nccl" in r["Name"].lower() or "rccl" in r["Name"].lower()]
print("RCCL kernels:", rccl)
print("ReduceScatter kernels:", [n for n, _ in rccl if "reducescatter" in n.lower().replace("_", "")])
PY
