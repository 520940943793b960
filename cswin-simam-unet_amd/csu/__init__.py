"""csu -- MI355X-native CSWin-(SimAM-)UNet training path.

Drop-in for the model/training API of TrungMasterChef/CSWin-SimAM-UNet
(train_cswinunet_segmentation.py, train_unet_segmentation.py): same class/function names,
constructor arguments and state_dict keys; compute runs in hand-written gfx950 kernels
(libcsu_hip.so, C ABI in include/csu.h).  Import with ``cswin-simam-unet_amd`` on sys.path.
"""
from .model import (CARAFE, CARAFE4, CSWinBlock, CSWinTransformer, DropPath, LePEAttention, Merge_Block, Mlp,
                    img2windows, windows2img)
from .simam import SimAM, simam
from .unet import DoubleConv, Down, UNet, Up
from .train import (bce_loss, dice_coefficient, evaluate_model, iou_score, make_optimizer, make_scheduler,
                    train_model, train_step)
from .optim import FusedAdam, FusedAdamW
from . import rng
from .rng import manual_seed

__all__ = ["UNet", "DoubleConv", "Down", "Up", "CARAFE", "CARAFE4", "CSWinBlock", "CSWinTransformer", "DropPath", "LePEAttention", "Merge_Block", "Mlp",
           "img2windows", "windows2img", "SimAM", "simam", "bce_loss", "dice_coefficient", "evaluate_model",
           "iou_score", "make_optimizer", "make_scheduler", "train_model", "train_step", "FusedAdamW", "FusedAdam",
           "rng", "manual_seed"]
