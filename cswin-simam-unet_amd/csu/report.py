"""Reporting and checkpointing around the training loop (train_cswinunet_segmentation.py
cswin:990-1071): the model ``.pth`` save (cswin:992), ``plot_metrics`` (cswin:1005-1049),
``save_metrics_to_csv`` (cswin:1052-1071) -- same file names, figure layout and CSV columns --
plus what the reference lacks: a resumable training checkpoint (model + optimizer + LR scheduler
+ epoch + history).  Under torch.distributed only rank 0 writes files."""
from __future__ import annotations

import csv
import os
from typing import Dict, List, Optional

import torch
import torch.distributed as dist

CSV_COLUMNS = ["Epoch", "Train_Loss", "Train_Dice", "Train_IoU", "Test_Loss", "Test_Dice", "Test_IoU", "Learning_Rate"]
HISTORY_KEYS = ["train_loss", "train_dice", "train_iou", "test_loss", "test_dice", "test_iou", "learning_rates"]


def _rank0() -> bool:
    return not (dist.is_available() and dist.is_initialized()) or dist.get_rank() == 0


def _unwrap(model):
    return getattr(model, "module", model)   # DistributedDataParallel -> the model


def save_metrics_to_csv(history: Dict[str, List[float]], path: str = "cswinunet_training_metrics.csv") -> Optional[str]:
    """One row per epoch: the reference's columns and number formats (6 decimals, lr 8)."""
    if not _rank0():
        return None
    with open(path, "w", newline="", encoding="utf-8") as f:
        w = csv.writer(f)
        w.writerow(CSV_COLUMNS)
        for i in range(len(history["train_loss"])):
            w.writerow([i + 1] + [f"{history[k][i]:.6f}" for k in HISTORY_KEYS[:6]] +
                       [f"{history['learning_rates'][i]:.8f}"])
    return path


def load_metrics_csv(path: str) -> Dict[str, List[float]]:
    """Inverse of save_metrics_to_csv (history dict with the reference's keys)."""
    hist = {k: [] for k in HISTORY_KEYS}
    with open(path, newline="", encoding="utf-8") as f:
        r = csv.reader(f)
        if next(r) != CSV_COLUMNS:
            raise ValueError(f"{path}: not a training-metrics CSV (columns {CSV_COLUMNS})")
        for row in r:
            for k, v in zip(HISTORY_KEYS, row[1:]):
                hist[k].append(float(v))
    return hist


def plot_metrics(history: Dict[str, List[float]], path: str = "cswinunet_training_metrics.png", dpi: int = 300):
    """2 x 2 figure: Loss, Dice, IoU (train blue / test red) and the learning rate (log scale)."""
    if not _rank0():
        return None
    import matplotlib
    matplotlib.use("Agg")
    import matplotlib.pyplot as plt
    epochs = range(1, len(history["train_loss"]) + 1)
    fig, axes = plt.subplots(2, 2, figsize=(16, 12))
    axes = axes.flatten()
    for ax, key, title in zip(axes[:3], ("loss", "dice", "iou"), ("Loss", "Dice Coefficient", "IoU Score")):
        ax.plot(epochs, history[f"train_{key}"], "b-", linewidth=2, label="Train")
        ax.plot(epochs, history[f"test_{key}"], "r-", linewidth=2, label="Test")
        ax.set_title(title, fontsize=14, fontweight="bold")
        ax.set_xlabel("Epoch")
        ax.set_ylabel({"loss": "Loss", "dice": "Dice", "iou": "IoU"}[key])
        ax.legend()
        ax.grid(True, alpha=0.3)
    axes[3].plot(epochs, history["learning_rates"], "g-", linewidth=2)
    axes[3].set_title("Learning Rate", fontsize=14, fontweight="bold")
    axes[3].set_xlabel("Epoch")
    axes[3].set_ylabel("Learning Rate")
    axes[3].set_yscale("log")
    axes[3].grid(True, alpha=0.3)
    plt.tight_layout()
    plt.savefig(path, dpi=dpi, bbox_inches="tight")
    plt.close(fig)
    return path


def save_model(model, path: str = "cswinunet_segmentation_model.pth") -> Optional[str]:
    """torch.save(model.state_dict(), path) (cswin:992): the reference's key/shape contract, so the
    file loads into the reference model and vice versa."""
    if not _rank0():
        return None
    torch.save(_unwrap(model).state_dict(), path)
    return path


def save_checkpoint(path: str, model, optimizer=None, scheduler=None, epoch: int = 0,
                    history: Optional[Dict[str, List[float]]] = None) -> Optional[str]:
    """Everything train_model needs to continue: model / optimizer / scheduler state, the number of
    finished epochs and the history so far.  Written atomically (tmp file + rename)."""
    if not _rank0():
        return None
    ck = {"model": _unwrap(model).state_dict(), "epoch": int(epoch),
          "history": {k: list(v) for k, v in (history or {}).items()}}
    if optimizer is not None:
        ck["optimizer"] = optimizer.state_dict()
    if scheduler is not None:
        ck["scheduler"] = scheduler.state_dict()
    tmp = path + ".tmp"
    torch.save(ck, tmp)
    os.replace(tmp, path)
    return path


def load_checkpoint(path: str, model, optimizer=None, scheduler=None, map_location=None):
    """Restore a save_checkpoint file into the given objects (weights_only load: nothing in the file
    is executed).  Returns (epochs finished, history).  A FusedAdamW with a device lr picks up the
    restored lr through sync_lr()."""
    ck = torch.load(path, map_location=map_location, weights_only=True)
    _unwrap(model).load_state_dict(ck["model"])
    if optimizer is not None and "optimizer" in ck:
        optimizer.load_state_dict(ck["optimizer"])
        if hasattr(optimizer, "sync_lr"):
            optimizer.sync_lr()
    if scheduler is not None and "scheduler" in ck:
        scheduler.load_state_dict(ck["scheduler"])
    return int(ck.get("epoch", 0)), {k: list(v) for k, v in ck.get("history", {}).items()}
