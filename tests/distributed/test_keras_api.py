"""Keras-style fit + Horovod Keras callbacks (``ewdml.parallel.keras``), the equivalent of the
reference's TF/Keras example ``tensorflow_mnist.py`` (callbacks ``:52-68``, rank-0 checkpoint
``:71-72``, ``fit`` ``:79``), on CPU Gloo worlds of 2 ranks."""
import os
import sys

import pytest
import torch

from .helpers import run_world

pytestmark = pytest.mark.slow

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def _example(rank, world, ckpt):
    sys.path.insert(0, ROOT)
    import horovod_keras_mnist as ex
    from ewdml.parallel import keras as hk

    lrs = []

    class Trace(hk.Callback):
        def on_batch_begin(self, batch, logs=None):
            lrs.append(self.optimizer.optimizer.param_groups[0]["lr"])

    orig_fit = hk.fit

    def fit(*a, callbacks=None, **kw):
        return orig_fit(*a, callbacks=list(callbacks) + [Trace()], **kw)

    hk.fit = fit
    try:
        model, hist = ex.main(["--epochs", "3", "--steps", "8", "--synthetic-size", "512",
                               "--batch-size", "16", "--warmup-epochs", "2", "--no-cuda",
                               "--checkpoint", ckpt])
    finally:
        hk.fit = orig_fit
    return {"params": [p.detach().clone() for p in model.parameters()],
            "history": hist.history, "lrs": lrs}


def test_keras_example_two_ranks(tmp_path):
    ckpt = str(tmp_path / "ckpt" / "checkpoint-{epoch}.pt")
    res = run_world(_example, 2, tmp_path / "w", args=(ckpt,))
    # broadcast at train begin + averaged gradients: identical replicas despite per-rank seeds
    for a, b in zip(res[0]["params"], res[1]["params"]):
        assert torch.equal(a, b)
    # MetricAverageCallback: the epoch logs are the ranks' mean, the same on both ranks
    assert res[0]["history"]["loss"] == res[1]["history"]["loss"]
    assert res[0]["history"]["accuracy"] == res[1]["history"]["accuracy"]
    assert len(res[0]["history"]["loss"]) == 3
    # LearningRateWarmupCallback: lr = init / size * (e * (size - 1) / warmup + 1),
    # e = epoch + (batch + 1) / steps, then init after the warm-up epochs
    init, size, warm, steps = 0.001 * 2, 2, 2, 8 // 2
    want = []
    for epoch in range(3):
        for b in range(steps):
            e = epoch + (b + 1) / steps
            want.append(init / size * (e * (size - 1) / warm + 1) if epoch < warm else init)
    assert res[0]["lrs"] == pytest.approx(want, rel=1e-12)
    assert res[0]["lrs"] == res[1]["lrs"]
    assert res[0]["lrs"][warm * steps - 1] == pytest.approx(init)  # reaches init_lr at the end
    # ModelCheckpoint on rank 0 only: one file per epoch, the last one = the final weights
    files = sorted(os.listdir(tmp_path / "ckpt"))
    assert files == [f"checkpoint-{e}.pt" for e in (1, 2, 3)]
    last = torch.load(tmp_path / "ckpt" / "checkpoint-3.pt", weights_only=True)
    for p, (k, v) in zip(res[0]["params"], last.items()):
        assert torch.equal(p, v), k


def _warmup_momentum(rank, world, lr_in_velocity=False):
    from ewdml.parallel import horovod as hvd
    from ewdml.parallel import keras as hk

    hvd.init(backend="gloo")
    torch.manual_seed(0)
    model = torch.nn.Linear(4, 2)
    opt = torch.optim.SGD(model.parameters(), lr=0.1, momentum=0.9)
    if lr_in_velocity:  # a Keras-style optimizer (v = m v - lr g): Horovod's correction applies
        opt.lr_in_velocity = True
    seen = []

    class Probe(hk.Callback):
        def on_batch_begin(self, batch, logs=None):
            g = opt.param_groups[0]
            seen.append((g["lr"], g["momentum"]))

    warm = hk.LearningRateWarmupCallback(initial_lr=0.4, warmup_epochs=1, steps_per_epoch=4)
    data = iter([(torch.randn(8, 4), torch.randint(0, 2, (8,))) for _ in range(8)])
    hk.fit(model, data, hvd.DistributedOptimizer(opt, model.named_parameters()),
           torch.nn.functional.cross_entropy, epochs=2, steps_per_epoch=4,
           callbacks=[warm, Probe()], verbose=0)
    return {"seen": seen, "final": opt.param_groups[0]["lr"], "mom": opt.param_groups[0]["momentum"]}


def _warmup_keras_style(rank, world):
    return _warmup_momentum(rank, world, lr_in_velocity=True)


@pytest.mark.parametrize("keras_style", [False, True])
def test_lr_warmup_momentum_correction(tmp_path, keras_style):
    """Momentum correction only for an optimizer whose lr sits inside the velocity (Keras SGD);
    torch.optim.SGD (p -= lr * buf) gets the plain warm-up: an lr change already rescales it."""
    res = run_world(_warmup_keras_style if keras_style else _warmup_momentum, 2, tmp_path)
    seen = res[0]["seen"]
    lrs = [0.4 / 2 * ((b + 1) / 4 * (2 - 1) / 1 + 1) for b in range(4)]
    old = [0.1] + lrs[:-1]
    for b in range(4):  # warm-up batches: lr and momentum * new / old for that batch only
        assert seen[b][0] == pytest.approx(lrs[b])
        want = 0.9 * lrs[b] / old[b] if keras_style else 0.9
        assert seen[b][1] == pytest.approx(want)
    for b in range(4, 8):  # after warm-up: initial_lr, momentum restored
        assert seen[b] == (pytest.approx(0.4), pytest.approx(0.9))
    assert res[0]["final"] == pytest.approx(0.4) and res[0]["mom"] == 0.9


def _metric_avg(rank, world):
    from ewdml.parallel import horovod as hvd
    from ewdml.parallel import keras as hk

    hvd.init(backend="gloo")
    logs = {"loss": 1.0 + rank, "accuracy": 0.5 * rank, "name": "x"}
    hk.MetricAverageCallback().on_epoch_end(0, logs)
    return logs


def test_metric_average_callback(tmp_path):
    res = run_world(_metric_avg, 3, tmp_path)
    for r in res:
        assert r["loss"] == pytest.approx(2.0) and r["accuracy"] == pytest.approx(0.5)
        assert r["name"] == "x"
