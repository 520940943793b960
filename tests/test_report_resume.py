"""Reporting and checkpoint/resume around train_model (cswin:751-841, 990-1071): CSV columns and
formats of save_metrics_to_csv, the metrics figure, and a resumed run that reproduces an
uninterrupted one (model, optimizer, ReduceLROnPlateau state and history).  CPU: a tiny torch
model stands in for the network (the loop and the checkpoint are model-agnostic); the csu model
with FusedAdamW is covered by tests/test_gpu_train.py."""
import csv
import os

import numpy as np
import torch
import torch.nn as nn

from csu import report
from csu.data import ellipse_batch
from csu.train import bce_loss, make_scheduler, train_model


def _net():
    torch.manual_seed(0)
    return nn.Sequential(nn.Conv2d(3, 6, 3, padding=1), nn.ReLU(), nn.Conv2d(6, 1, 1), nn.Sigmoid())


class _Stream:
    """Loader yielding `per_epoch` fresh batches of a fixed rng stream per epoch."""

    def __init__(self, batches, per_epoch):
        self.batches, self.per_epoch, self.pos = batches, per_epoch, 0

    def __iter__(self):
        out = self.batches[self.pos:self.pos + self.per_epoch]
        self.pos += self.per_epoch
        return iter(out)


def _data(epochs, per_epoch=3):
    rng = np.random.default_rng(1234)
    train = [ellipse_batch(rng, 2, 16) for _ in range(epochs * per_epoch)]
    test = [ellipse_batch(np.random.default_rng(99), 4, 16)]
    return train, test


def _run(num_epochs, train, test, start_pos=0, ckpt=None, resume=None):
    m = _net()
    opt = torch.optim.AdamW(m.parameters(), lr=1e-2, weight_decay=1e-4)
    sch = make_scheduler(opt, patience=0)
    loader = _Stream(train, 3)
    loader.pos = start_pos
    h = train_model(m, loader, test, bce_loss, opt, sch, torch.device("cpu"), num_epochs=num_epochs, verbose=False,
                    checkpoint_path=ckpt, resume_from=resume)
    return m, opt, sch, h


def test_resume_reproduces_uninterrupted_run(tmp_path):
    train, test = _data(4)
    m_ref, opt_ref, sch_ref, h_ref = _run(4, train, test)
    ck = str(tmp_path / "ck.pt")
    _run(2, train, test, ckpt=ck)
    m, opt, sch, h = _run(4, train, test, start_pos=6, resume=ck)
    assert h == h_ref
    for a, b in zip(m.parameters(), m_ref.parameters()):
        assert torch.equal(a, b)
    assert sch.state_dict()["num_bad_epochs"] == sch_ref.state_dict()["num_bad_epochs"]
    assert opt.param_groups[0]["lr"] == opt_ref.param_groups[0]["lr"]


def test_metrics_csv_and_plot(tmp_path):
    train, test = _data(3)
    *_, h = _run(3, train, test)
    p = report.save_metrics_to_csv(h, str(tmp_path / "m.csv"))
    with open(p, newline="") as f:
        rows = list(csv.reader(f))
    assert rows[0] == ["Epoch", "Train_Loss", "Train_Dice", "Train_IoU", "Test_Loss", "Test_Dice", "Test_IoU",
                       "Learning_Rate"]                                                       # cswin:1058-1059
    assert [r[0] for r in rows[1:]] == ["1", "2", "3"]
    assert rows[1][1] == f"{h['train_loss'][0]:.6f}" and rows[1][7] == f"{h['learning_rates'][0]:.8f}"
    back = report.load_metrics_csv(p)
    for k in h:
        np.testing.assert_allclose(back[k], h[k], atol=1e-6 if k != "learning_rates" else 1e-8)
    png = report.plot_metrics(h, str(tmp_path / "m.png"), dpi=40)
    assert os.path.getsize(png) > 1000


def test_save_model_is_a_plain_state_dict(tmp_path):
    m = _net()
    p = report.save_model(m, str(tmp_path / "w.pth"))
    sd = torch.load(p, weights_only=True)
    assert list(sd) == list(m.state_dict())
