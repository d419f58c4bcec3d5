"""The reference's Horovod TF/Keras MNIST example (``tensorflow_mnist.py``) on the ewdml stack.

TensorFlow is not part of an MI355X PyTorch-ROCm build, so the same program is written against
``ewdml.parallel.keras`` (a Keras-style ``fit`` with Horovod's Keras callbacks) and the Horovod
API: init and pin the device to the local rank (``:5-15``), MNIST with repeat / shuffle / batch
128 (``:17-24``), the Conv32-Conv64-MaxPool-Dropout-Dense128-Dropout-Dense10 CNN (``:26-35``,
``models.KerasMnistCNN``), Adam at ``0.001 * size`` (``:38-39``) wrapped in
``DistributedOptimizer(backward_passes_per_step=1)`` with gradient averaging (``:42-43``), the
broadcast / metric-average / LR-warmup callbacks (``:52-68``), checkpoints on rank 0 only
(``:71-72``) and ``fit(steps_per_epoch=500 // size, epochs=24)`` (``:79``).

    torchrun --standalone --nproc-per-node 2 horovod_keras_mnist.py --epochs 3
"""
import argparse
import os

import torch
import torch.nn.functional as F

import ewdml as hvd
from ewdml.data import DeviceLoader, load_dataset
from ewdml.models import KerasMnistCNN
from ewdml.parallel import keras as hk


def parse(argv=None):
    p = argparse.ArgumentParser(description="Horovod Keras MNIST example (ewdml)")
    p.add_argument("--epochs", type=int, default=24)
    p.add_argument("--steps", type=int, default=500, help="steps per epoch before / size")
    p.add_argument("--batch-size", type=int, default=128)
    p.add_argument("--base-lr", type=float, default=0.001)
    p.add_argument("--warmup-epochs", type=int, default=3)
    p.add_argument("--data-dir", default=None, help="MNIST IDX directory (default: synthetic)")
    p.add_argument("--synthetic-size", type=int, default=0)
    p.add_argument("--compression", default="none",
                   choices=["none", "fp16", "bf16", "qsgd", "topk", "topk_qsgd"])
    p.add_argument("--checkpoint", default="./checkpoint-{epoch}.pt")
    p.add_argument("--no-cuda", action="store_true")
    p.add_argument("--seed", type=int, default=0)
    return p.parse_args(argv)


def main(argv=None):
    args = parse(argv)
    cuda = not args.no_cuda and torch.cuda.is_available()
    hvd.init(backend=None if cuda else "gloo")
    device = torch.device("cuda", hvd.local_rank()) if cuda else torch.device("cpu")
    torch.manual_seed(args.seed + hvd.rank())  # different init per rank: the broadcast syncs it

    x, y, info = load_dataset("MNIST", args.data_dir, train=True,
                              synthetic_size=args.synthetic_size, seed=args.seed, device=device)
    loader = DeviceLoader(x, y, info, args.batch_size, hvd.rank(), hvd.size(), seed=args.seed)

    def batches():  # dataset.repeat().shuffle(10000).batch(128): an endless reshuffled stream
        while True:
            yield loader.next()

    model = KerasMnistCNN().to(device)
    scaled_lr = args.base_lr * hvd.size()
    opt = torch.optim.Adam(model.parameters(), lr=scaled_lr)
    comp = {"none": hvd.Compression.none, "fp16": hvd.Compression.fp16,
            "bf16": hvd.Compression.bf16, "qsgd": hvd.Compression.qsgd(),
            "topk": hvd.Compression.topk(0.01),
            "topk_qsgd": hvd.Compression.topk_qsgd(0.01)}[args.compression]
    opt = hvd.DistributedOptimizer(opt, model.named_parameters(), compression=comp,
                                   backward_passes_per_step=1, op=hvd.Average)

    callbacks = [
        hk.callbacks.BroadcastGlobalVariablesCallback(0),
        hk.callbacks.MetricAverageCallback(),
        hk.callbacks.LearningRateWarmupCallback(initial_lr=scaled_lr,
                                                warmup_epochs=args.warmup_epochs, verbose=1),
    ]
    if hvd.rank() == 0:  # checkpoints on worker 0 only
        d = os.path.dirname(args.checkpoint)
        if d:
            os.makedirs(d, exist_ok=True)
        callbacks.append(hk.ModelCheckpoint(args.checkpoint))
    verbose = 1 if hvd.rank() == 0 else 0
    hist = hk.fit(model, batches(), opt, F.cross_entropy, epochs=args.epochs,
                  steps_per_epoch=max(1, args.steps // hvd.size()), callbacks=callbacks,
                  verbose=verbose, device=device)
    return model, hist


if __name__ == "__main__":
    main()
