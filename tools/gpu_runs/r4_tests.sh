# Round 4: the GPU test suite (optionally a subset: TESTS / KEXPR), then smoke
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r4_tests
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest ${TESTS:-tests} -m gpu -x -v --timeout 200 --timeout-method thread -p no:cacheprovider ${KEXPR:+-k "$KEXPR"} > gpurun_out/r4_tests/pytest.log 2>&1
rc=$?; echo "pytest rc=$rc $(tail -1 gpurun_out/r4_tests/pytest.log)"; grep -E "FAILED|Error" gpurun_out/r4_tests/pytest.log | head -20; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r4_tests/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc $(tail -1 gpurun_out/r4_tests/smoke.log)"; exit $rc
