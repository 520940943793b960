# round-4: the graph-reproducibility test with per-parameter diagnostics, then the rest of the GPU suite
set -o pipefail
O=gpurun_out/r06k; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py -q -k "reproducible" --timeout 300 --timeout-method thread > $O/repro.log 2>&1; echo "repro rc=$?"
grep -E "passed|failed|AssertionError|assert not diff" $O/repro.log | head -5
timeout -k 10 600 python -u -m pytest tests/test_gpu_train.py tests/test_gpu_unet.py -q --deselect "tests/test_gpu_train.py::test_graph_replays_bitwise_reproducible" --timeout 300 --timeout-method thread > $O/rest.log 2>&1 || { echo REST_FAIL; tail -30 $O/rest.log; exit 1; }
tail -1 $O/rest.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo SMOKE_FAIL; tail -20 $O/smoke.log; exit 1; }
echo ALL_OK
