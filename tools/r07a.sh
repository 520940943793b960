# round 5, first GPU call: the full -m gpu suite (determinism fix, full-size config tests), the
# RCCL two-ranks-on-one-GPU probe, a headline bench line.  Stops after any crash / timeout.
O=gpurun_out/r07a; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/gpu_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 120 python -u tools/probes/rccl_one_gpu.py > $O/rccl_probe.log 2>&1
rc=$?; echo "probe rc=$rc"; tail -4 $O/rccl_probe.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err
rc=$?; echo "bench rc=$rc"; tail -c 400 $O/bench.json
