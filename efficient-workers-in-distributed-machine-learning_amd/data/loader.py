"""Device-resident loader with a rank-sharded sampler and GPU-side augmentation.

``DeviceLoader`` holds the uint8 dataset in device memory.  Each epoch draws one permutation from
a generator seeded with (seed, epoch) -- identical on every rank -- and rank r takes positions
r, r+W, r+2W, ... truncated so that every rank gets exactly the same number of full batches
(``torch.utils.data.DistributedSampler`` semantics with drop_last).  Batches are gathered by index,
converted to float, optionally augmented (CIFAR: reflect-pad 4 / random crop 32 / h-flip, as
``util.py:38-48``) and normalised, all on the device.

``fused=True`` (GPU training loaders): the whole batch is built by ONE kernel
(``ops.make_batch``, ``ops/csrc/data.hip``) into static output buffers, with the batch position
kept on the device so the launch can be captured in the training step's HIP graph
(:meth:`emit`); the host only tracks the position to roll epochs over (:meth:`begin_step`).
Augmentation draws then come from a counter hash instead of ``torch.Generator``.
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
                 seed=0, device=None, channels_last=False, drop_last=True, fused=False,
                 out_dtype=torch.float32):
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
        self.fused = bool(fused) and drop_last and self.device.type == "cuda" and \
            self.x.dim() == 4 and self.x.dtype == torch.uint8 and self.x.shape[1] <= 4
        if self.fused:
            from .. import ops

            ops.require()
            self.x = self.x.contiguous()
            self._mean_l = [float(v) for v in info["mean"]]
            self._istd_l = [1.0 / float(v) for v in info["std"]]
            B, (C, H, W) = batch_size, self.x.shape[1:]
            fmt = torch.channels_last if channels_last else torch.contiguous_format
            self.bx = torch.empty((B, C, H, W), dtype=out_dtype, device=self.device,
                                  memory_format=fmt)
            self.by = torch.empty(B, dtype=torch.int64, device=self.device)
            self._state = torch.zeros(2, dtype=torch.int64, device=self.device)  # pos, epoch
            self._done = torch.zeros(ops.TICKET_INTS, dtype=torch.int32, device=self.device)
            self._perm = torch.empty(self.per_rank, dtype=torch.int64, device=self.device)
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
        if self.fused:  # device-side state read by the (possibly graph-captured) batch kernel
            self._perm.copy_(self._idx)
            self._state[0].zero_()
            self._state[1].fill_(epoch)

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

    def begin_step(self):
        """Roll over to the next epoch if this one is exhausted (host side; same on every rank)."""
        if self._pos >= self.batches_per_epoch:
            self._start_epoch(self.epoch + 1)

    def emit(self, defer=False):
        """(fused) Launch the batch kernel for the device-side position and return the static
        (x, y) buffers; graph-capturable.  The caller advances the host position (:meth:`advance`).

        ``defer``: no launch -- the buffers carry ``_ew_batch`` (this loader) and the consumer
        either forms the batch in its own first launch (ops/lenet.py: the LeNet conv launch,
        :meth:`batch_args`) or calls :meth:`flush` before reading them."""
        if defer and self.batch_fusable():
            self._deferred = True
            self.bx._ew_batch = self
            return self.bx, self.by
        # (a deferral left over from an aborted capture never ran: dropped, not launched)
        self._deferred = False
        self.bx._ew_batch = None
        self._launch()
        return self.bx, self.by

    def _launch(self):
        from .. import ops

        ops.make_batch(self.x, self.y, self._perm, self._state, self._done, self.bx, self.by,
                       self._mean_l, self._istd_l, pad=4, augment=self.augment,
                       seed=self.seed * 7919 + 17, rank=self.rank)

    def batch_fusable(self) -> bool:
        """A consumer may form this loader's batch itself: fp32 NCHW, one channel, no
        augmentation (the LeNet conv launch's gather)."""
        return (self.fused and not self.augment and self.x.shape[1] == 1
                and self.bx.dtype == torch.float32 and self.bx.is_contiguous())

    def take_deferred(self):
        """(consumer) The pending batch's kernel arguments, or None; the batch is then the
        consumer's to form."""
        if not getattr(self, "_deferred", False):
            return None
        self._deferred = False
        self.bx._ew_batch = None
        return (self.x, self.y, self._perm, self._state, self._done, self._mean_l[0],
                self._istd_l[0])

    def flush(self):
        """Launch a deferred batch kernel (a consumer that cannot form the batch)."""
        if getattr(self, "_deferred", False):
            self._deferred = False
            self.bx._ew_batch = None
            self._launch()

    def advance(self):
        self._pos += 1

    def seek(self, pos):
        """Position within the current epoch (resume)."""
        self._pos = int(pos)
        if self.fused:
            self._state[0].fill_(self._pos)

    def next(self, static=False):
        """Next batch; rolls over to the next epoch (same count on every rank).  Fused loaders
        return their static buffers when ``static`` (overwritten by the next call), else copies."""
        self.begin_step()
        if self.fused:
            x, y = self.emit()
            self.advance()
            return (x, y) if static else (x.clone(memory_format=torch.preserve_format), y.clone())
        s = self._pos * self.batch_size
        self._pos += 1
        return self._make(self._idx[s:s + self.batch_size])

    def __iter__(self):
        """The rest of the current epoch (a fresh epoch if the current one is exhausted)."""
        if self._pos >= self.batches_per_epoch:
            self._start_epoch(self.epoch + 1)
        for _ in range(self.batches_per_epoch - self._pos):
            yield self.next()


def fused_draws(seed, rank, epoch, slot, pad=4):
    """(dy, dx, flip) of the fused batch kernel for one sample slot (== ``csrc/data.hip``)."""
    from ..compress.rng import M32, mix32_int

    a = mix32_int((seed * 0x9E3779B9 + rank) & M32)
    b = mix32_int((epoch * 0x85EBCA6B + slot) & M32)
    h = mix32_int(a ^ b)
    span = 2 * pad + 1
    return (h & 0xFF) % span, ((h >> 8) & 0xFF) % span, (h >> 16) & 1


def reference_fused_batch(x, y, perm, pos, batch, mean, inv_std, augment, seed, rank, epoch,
                          pad=4):
    """Torch oracle of ``ops.make_batch`` (fp32 NCHW; the kernel's arithmetic, same draws)."""
    idx = perm[pos * batch:(pos + 1) * batch]
    xs = x.index_select(0, idx).to(torch.float32)
    n, c, h, w = xs.shape
    if augment:
        xp = F.pad(xs, (pad, pad, pad, pad), mode="reflect")
        out = torch.empty_like(xs)
        for b in range(n):
            dy, dx, flip = fused_draws(seed, rank, epoch, pos * batch + b, pad)
            crop = xp[b, :, dy:dy + h, dx:dx + w]
            out[b] = crop.flip(-1) if flip else crop
        xs = out
    m = torch.tensor(mean, dtype=torch.float32, device=xs.device).view(1, -1, 1, 1)
    s = torch.tensor(inv_std, dtype=torch.float32, device=xs.device).view(1, -1, 1, 1)
    return (xs * (1.0 / 255.0) - m) * s, y.index_select(0, idx)
