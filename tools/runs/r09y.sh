# gemm4 split-K for the 4096-token K = 1536 / 2048 shapes (G4_SPLITK 1, libcsu_hip.so) vs none (ab)
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "gemm or linear or model or split" > gpurun_out/r09y_tests.log 2>&1 || { tail -30 gpurun_out/r09y_tests.log; exit 1; }
tail -2 gpurun_out/r09y_tests.log
sed -e 's/r09x/r09y/g' tools/runs/r09x.sh > /tmp/r09y_shapes.sh
bash /tmp/r09y_shapes.sh || exit 1
bash tools/ab_1024.sh r09y gemm
