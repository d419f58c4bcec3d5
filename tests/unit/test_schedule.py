"""LR schedule: Horovod-style warmup (lr/W -> lr) and step decay."""
import pytest

import ewdml
from ewdml.runtime import Trainer


def test_lr_warmup_and_decay():
    cfg = ewdml.parse_args(["--device", "cpu", "--synthetic-size", "640", "--batch-size", "64",
                            "--lr", "0.1", "--lr-warmup-epochs", "2", "--lr-decay-epochs", "3,5",
                            "--lr-decay", "0.5", "--quiet", "--eval-freq", "0"])
    tr = Trainer(cfg)
    spe = len(tr.loader)
    assert tr.lr_at(0) == pytest.approx(0.1)  # world of 1: warmup starts at lr / 1
    tr.n_workers = 4
    assert tr.lr_at(0) == pytest.approx(0.025)
    assert tr.lr_at(spe) == pytest.approx(0.025 + 0.075 / 2)
    assert tr.lr_at(2 * spe) == pytest.approx(0.1)
    assert tr.lr_at(3 * spe) == pytest.approx(0.05)
    assert tr.lr_at(6 * spe) == pytest.approx(0.025)
