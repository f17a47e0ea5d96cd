# Deterministic mode on all models: determinism tests + embedding / BERT / MLP GPU tests.
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/det2
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "determin or bag or bert or mlp or big_model or layernorm or gelu" > gpurun_out/det2/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/det2/pytest.log)"; [ $rc -eq 0 ] || { grep -E "Error|assert|FAILED" gpurun_out/det2/pytest.log | head -20; exit $rc; }
