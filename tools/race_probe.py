"""Repeat the graphed-vs-eager comparison with side-stream weight gradients on and off."""
import os, sys
sys.path[:0] = [os.path.join(os.path.dirname(__file__), ".."), os.path.join(os.path.dirname(__file__), "..", "cswin-simam-unet_amd"),
                os.path.join(os.path.dirname(__file__), "..", "tests")]
import torch
from csu import ops
import test_gpu_model as T

for side in (True, False, True, False):
    ops.SIDE_WGRAD = side
    try:
        T.test_graphed_train_step_matches_eager()
        print("side", side, "OK", flush=True)
    except AssertionError as e:
        print("side", side, "FAIL", str(e).split("\n")[2:5], flush=True)
