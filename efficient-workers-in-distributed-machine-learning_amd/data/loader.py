"""Device-resident loader with a rank-sharded sampler and GPU-side augmentation.

``DeviceLoader`` holds the uint8 dataset in device memory.  Each epoch draws one permutation from
a generator seeded with (seed, epoch) -- identical on every rank -- and rank r takes positions
r, r+W, r+2W, ... truncated so that every rank gets exactly the same number of full batches
(``torch.utils.data.DistributedSampler`` semantics with drop_last).  Batches are gathered by index,
converted to float, optionally augmented (CIFAR: reflect-pad 4 / random crop 32 / h-flip, as
``util.py:38-48``) and normalised, all on the device.
"""
import torch
import torch.nn.functional as F


def augment_cifar(x: torch.Tensor, gen: torch.Generator = None, pad: int = 4) -> torch.Tensor:
    """Reflect-pad, random crop back to H x W, random horizontal flip; x float [N,C,H,W]."""
    n, c, h, w = x.shape
    xp = F.pad(x, (pad, pad, pad, pad), mode="reflect")
    dev = x.device
    dy = torch.randint(0, 2 * pad + 1, (n,), device=dev, generator=gen)
    dx = torch.randint(0, 2 * pad + 1, (n,), device=dev, generator=gen)
    flip = torch.rand(n, device=dev, generator=gen) < 0.5
    iy = dy[:, None] + torch.arange(h, device=dev)[None, :]  # [n, h]
    ix = dx[:, None] + torch.arange(w, device=dev)[None, :]  # [n, w]
    ix = torch.where(flip[:, None], ix.flip(1), ix)
    rows = xp.gather(2, iy[:, None, :, None].expand(n, c, h, xp.shape[3]))
    return rows.gather(3, ix[:, None, None, :].expand(n, c, h, w))


class DeviceLoader:
    def __init__(self, x, y, info, batch_size, rank=0, world=1, shuffle=True, augment=False,
                 seed=0, device=None, channels_last=False, drop_last=True):
        self.device = torch.device(device) if device is not None else x.device
        self.x = x.to(self.device)
        self.y = y.to(self.device)
        self.batch_size = batch_size
        self.rank, self.world = rank, world
        self.shuffle, self.augment, self.seed = shuffle, augment, seed
        self.channels_last = channels_last
        self.drop_last = drop_last
        mean = torch.tensor(info["mean"], dtype=torch.float32, device=self.device)
        std = torch.tensor(info["std"], dtype=torch.float32, device=self.device)
        self.mean = mean.view(1, -1, 1, 1)
        self.inv_std = (1.0 / std).view(1, -1, 1, 1)
        n = self.x.shape[0]
        per_rank = n // world
        self.batches_per_epoch = per_rank // batch_size if drop_last else -(-per_rank // batch_size)
        if self.batches_per_epoch == 0:
            raise ValueError(f"dataset of {n} samples is too small for {world} ranks x batch "
                             f"{batch_size}")
        self.per_rank = self.batches_per_epoch * batch_size if drop_last else per_rank
        self.epoch = 0
        self._gen = torch.Generator(device=self.device)
        self._idx = None
        self._pos = 0
        self._start_epoch(0)

    def _start_epoch(self, epoch):
        self.epoch = epoch
        n = self.x.shape[0]
        if self.shuffle:
            # generated on the device: no host round trip (a CPU permutation + copy would block
            # the host until the GPU drains, a bubble at every epoch start); the same seed gives
            # the same permutation on every rank
            g = torch.Generator(device=self.device).manual_seed(self.seed * 100003 + epoch)
            perm = torch.randperm(n, generator=g, device=self.device)
        else:
            perm = torch.arange(n, device=self.device)
        self._idx = perm[self.rank::self.world][:self.per_rank]
        self._gen.manual_seed(self.seed * 7919 + epoch * 31 + self.rank)
        self._pos = 0

    def __len__(self):
        return self.batches_per_epoch

    def set_epoch(self, epoch):
        self._start_epoch(epoch)

    def _make(self, idx):
        x = self.x.index_select(0, idx).to(torch.float32) * (1.0 / 255.0)
        if self.augment:
            x = augment_cifar(x, self._gen)
        x = (x - self.mean) * self.inv_std
        if self.channels_last:
            x = x.contiguous(memory_format=torch.channels_last)
        return x, self.y.index_select(0, idx)

    def next(self):
        """Next batch; rolls over to the next epoch (same count on every rank)."""
        if self._pos >= self.batches_per_epoch:
            self._start_epoch(self.epoch + 1)
        s = self._pos * self.batch_size
        self._pos += 1
        return self._make(self._idx[s:s + self.batch_size])

    def __iter__(self):
        """The rest of the current epoch (a fresh epoch if the current one is exhausted)."""
        if self._pos >= self.batches_per_epoch:
            self._start_epoch(self.epoch + 1)
        for _ in range(self.batches_per_epoch - self._pos):
            yield self.next()
