set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_unet.py tests/test_gpu_model.py -k "unet or bn or maxpool" -x -q --timeout 120 --timeout-method thread 2>&1 | tail -30
