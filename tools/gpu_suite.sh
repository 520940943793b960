# The -m gpu suite on the box, output under gpurun_out/$1/ (optional pytest -k filter as $2).
O=gpurun_out/$1; mkdir -p $O
K=${2:+-k "$2"}
eval timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread $K > $O/gpu_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -4 $O/gpu_tests.log; exit $rc
