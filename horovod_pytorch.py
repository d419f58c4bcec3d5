"""Horovod-style MNIST training on the ewdml API (no Horovod, no MPI).

Same flags and flow as the reference's ``horvod_pytorch.py``: init, pin the device to the local
rank, shard the data per rank, scale the LR by the world size (not for Adasum), broadcast the
initial parameters and optimizer state from rank 0, wrap the optimizer in
``DistributedOptimizer(compression=..., op=Average|Adasum, gradient_predivide_factor=...)``, train,
and average the test metrics across ranks with ``allreduce``.

    torchrun --standalone --nproc-per-node 2 horovod_pytorch.py --compression qsgd --epochs 1
"""
import argparse

import torch
import torch.nn.functional as F

import ewdml as hvd
from ewdml.data import DeviceLoader, load_dataset
from ewdml.models import MnistNet


def parse(argv=None):
    p = argparse.ArgumentParser(description="PyTorch MNIST Example (ewdml)")
    p.add_argument("--batch-size", type=int, default=64)
    p.add_argument("--test-batch-size", type=int, default=1000)
    p.add_argument("--epochs", type=int, default=10)
    p.add_argument("--lr", type=float, default=0.01)
    p.add_argument("--momentum", type=float, default=0.5)
    p.add_argument("--no-cuda", action="store_true", default=False)
    p.add_argument("--seed", type=int, default=42)
    p.add_argument("--log-interval", type=int, default=10)
    p.add_argument("--fp16-allreduce", action="store_true", default=False)
    p.add_argument("--use-adasum", action="store_true", default=False)
    p.add_argument("--gradient-predivide-factor", type=float, default=1.0)
    p.add_argument("--data-dir", default=None, help="MNIST IDX directory (default: synthetic)")
    p.add_argument("--compression", default="qsgd",
                   choices=["none", "fp16", "bf16", "qsgd", "topk", "topk_qsgd"],
                   help="the reference wires its QSGDCompressor (horvod_pytorch.py:194)")
    p.add_argument("--max-steps", type=int, default=None)
    p.add_argument("--synthetic-size", type=int, default=0)
    return p.parse_args(argv)


def metric_average(val, name):
    return float(hvd.allreduce(torch.tensor(float(val)), name=name))


def main(argv=None):
    args = parse(argv)
    args.cuda = not args.no_cuda and torch.cuda.is_available()
    hvd.init(backend=None if args.cuda else "gloo")
    torch.manual_seed(args.seed)
    device = torch.device("cuda", hvd.local_rank()) if args.cuda else torch.device("cpu")

    x, y, info = load_dataset("MNIST", args.data_dir, train=True,
                              synthetic_size=args.synthetic_size, seed=args.seed, device=device)
    tx, ty, _ = load_dataset("MNIST", args.data_dir, train=False,
                             synthetic_size=args.synthetic_size // 5 if args.synthetic_size else 0,
                             seed=args.seed, device=device)
    train = DeviceLoader(x, y, info, args.batch_size, hvd.rank(), hvd.size(), seed=args.seed)
    test = DeviceLoader(tx, ty, info, min(args.test_batch_size, tx.shape[0]), hvd.rank(),
                        hvd.size(), shuffle=False, drop_last=False)

    model = MnistNet().to(device)
    lr_scaler = hvd.size() if not args.use_adasum else 1
    optimizer = torch.optim.SGD(model.parameters(), lr=args.lr * lr_scaler,
                                momentum=args.momentum)
    hvd.broadcast_parameters(model.state_dict(), root_rank=0)
    hvd.broadcast_optimizer_state(optimizer, root_rank=0)
    if args.compression == "qsgd":
        compression = hvd.Compression.qsgd()
    elif args.fp16_allreduce:
        compression = hvd.Compression.fp16
    else:
        compression = args.compression
    optimizer = hvd.DistributedOptimizer(
        optimizer, named_parameters=model.named_parameters(), compression=compression,
        op=hvd.Adasum if args.use_adasum else hvd.Average,
        gradient_predivide_factor=args.gradient_predivide_factor)

    step = 0
    for epoch in range(1, args.epochs + 1):
        model.train()
        train.set_epoch(epoch)
        for batch_idx, (data, target) in enumerate(train):
            optimizer.zero_grad()
            loss = F.nll_loss(model(data), target)
            loss.backward()
            optimizer.step()
            step += 1
            if batch_idx % args.log_interval == 0 and hvd.rank() == 0:
                print(f"Train Epoch: {epoch} [{batch_idx * len(data)}/{train.per_rank}]\t"
                      f"Loss: {loss.item():.6f}", flush=True)
            if args.max_steps and step >= args.max_steps:
                break
        model.eval()
        test_loss = test_acc = 0.0
        n = 0
        with torch.no_grad():
            for data, target in test:
                out = model(data)
                test_loss += float(F.nll_loss(out, target, reduction="sum"))
                test_acc += float((out.argmax(1) == target).sum())
                n += target.shape[0]
        test_loss = metric_average(test_loss / n, "avg_loss")
        test_acc = metric_average(test_acc / n, "avg_accuracy")
        if hvd.rank() == 0:
            print(f"\nTest set: Average loss: {test_loss:.4f}, Accuracy: {100 * test_acc:.2f}%\n",
                  flush=True)
        if args.max_steps and step >= args.max_steps:
            break
    return {"test_loss": test_loss, "test_acc": test_acc, "steps": step}


if __name__ == "__main__":
    main()
