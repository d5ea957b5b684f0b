# GPU call script (gpurun): the round-end gate on the final tree -- the whole GPU suite, smoke() and the bench line.
set -o pipefail
cd $GRAFT_REPO_ROOT
O=gpurun_out/r4v; mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1; rc=$?; tail -2 $O/pytest.log; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; echo "smoke rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.log 2>&1; rc=$?; grep -o '"value": [0-9.]*\|"ok": [a-z]*' $O/bench.log | head -3 | tr '\n' ' '; echo "bench rc=$rc"
