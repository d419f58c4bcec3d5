"""Atomic rank-0 checkpoints, resume, and the reference's evaluator-visible ``model_step_`` file.

The reference saves ``state_dict()`` every ``--eval-freq`` steps from *every* worker to the same
path ``train_dir + "model_step_"`` (``distributed_worker.py:237-238, 392-398``: a write/read race
with the evaluator) and has no resume.  Here rank 0 alone writes
``{ckpt_dir}/step_{N}.pt`` = {model state, optimizer state (momentum / Adam moments), error-feedback
residual, step, epoch, RNG states, config} through write-to-temp + ``os.replace``, then points
``latest`` at it.  ``model_step_`` (a plain ``state_dict``, loadable by the reference evaluator and by
``distributed_evaluator.py``) is written the same atomic way when ``legacy`` is on.
"""
import os
import tempfile

import torch


def _atomic_save(obj, path):
    d = os.path.dirname(os.path.abspath(path))
    os.makedirs(d, exist_ok=True)
    fd, tmp = tempfile.mkstemp(dir=d, prefix="tmp_ckpt_", suffix=".part")
    os.close(fd)
    try:
        torch.save(obj, tmp)
        os.replace(tmp, path)
    finally:
        if os.path.exists(tmp):
            os.remove(tmp)


def _cpu(x):
    if torch.is_tensor(x):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _cpu(v) for k, v in x.items()}
    return x


def save(ckpt_dir, step, model, optimizer, epoch=0, extra=None, legacy_dir=None, keep=3,
         model_state=None):
    state = {
        "step": int(step),
        "epoch": int(epoch),
        "model": _cpu(model_state if model_state is not None else model.state_dict()),
        "optimizer": _cpu(optimizer.state_dict()) if optimizer is not None else None,
        "rng_cpu": torch.get_rng_state(),
        "rng_cuda": torch.cuda.get_rng_state_all() if torch.cuda.is_available() else None,
        "extra": _cpu(extra or {}),
    }
    path = os.path.join(ckpt_dir, f"step_{step}.pt")
    _atomic_save(state, path)
    link = os.path.join(ckpt_dir, "latest")
    tmp = link + ".tmp"
    if os.path.lexists(tmp):
        os.remove(tmp)
    os.symlink(os.path.basename(path), tmp)
    os.replace(tmp, link)
    if legacy_dir is not None:
        _atomic_save(state["model"], os.path.join(legacy_dir, "model_step_"))
    if keep:
        olds = sorted((f for f in os.listdir(ckpt_dir) if f.startswith("step_") and
                       f.endswith(".pt")), key=lambda f: int(f[5:-3]))
        for f in olds[:-keep]:
            os.remove(os.path.join(ckpt_dir, f))
    return path


def latest(ckpt_dir):
    link = os.path.join(ckpt_dir, "latest")
    if os.path.exists(link):
        return os.path.realpath(link)
    return None


def load(path, map_location="cpu"):
    """Load a checkpoint written by :func:`save` (tensors and plain containers only)."""
    return torch.load(path, map_location=map_location, weights_only=True)
