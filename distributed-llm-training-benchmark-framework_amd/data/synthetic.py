"""Synthetic token data (reference: ``SyntheticDataset`` + DataLoader, train_harness.py:138-150,
:304-325).

* ``SyntheticDataset``: a fixed ``randint(0, vocab, (size, seq_len))`` int64 table from a private
  generator seeded with ``seed`` (the reference re-seeds the *global* RNG instead; we do not touch
  global state).
* Sampling reproduces the reference: DDP/FSDP at world_size > 1 use a DistributedSampler-style
  shuffled, padded, rank-strided permutation (seed 0, epoch never advanced - the reference never
  calls ``set_epoch``); ZeRO paths and world_size 1 use a plain shuffle that is identical on every
  rank (in the reference the DataLoader shuffle draws from the global RNG right after the dataset
  re-seeded it to 42, so all ZeRO ranks see the same batches).
* ``DeviceBatcher`` keeps the whole table resident in HBM (16 MB for 1000 x 2048) and gathers each
  micro-batch on the GPU - no per-step host->device copy.  ``HostBatcher`` reproduces the reference's
  pinned-memory DataLoader + ``non_blocking`` H2D copy.
"""
import torch


class SyntheticDataset:
    def __init__(self, vocab_size: int = 32000, seq_len: int = 2048, size: int = 1000, seed: int = 42):
        g = torch.Generator().manual_seed(seed)
        self.data = torch.randint(0, vocab_size, (size, seq_len), generator=g, dtype=torch.int64)
        self.size, self.seq_len, self.vocab_size = size, seq_len, vocab_size

    def __len__(self):
        return self.size

    def __getitem__(self, i):
        return self.data[i]


def epoch_indices(n: int, world: int, rank: int, distributed: bool, seed: int = 0, epoch: int = 0):
    g = torch.Generator().manual_seed(seed + epoch)
    perm = torch.randperm(n, generator=g)
    if not distributed or world == 1:
        return perm
    total = (n + world - 1) // world * world
    if total > n:
        perm = torch.cat([perm, perm[: total - n]])
    return perm[rank:total:world]


class _Batcher:
    def __init__(self, ds: SyntheticDataset, batch_size: int, world: int, rank: int, distributed: bool,
                 shuffle_seed: int):
        self.ds, self.B, self.world, self.rank = ds, batch_size, world, rank
        self.distributed, self.seed = distributed, shuffle_seed
        self.epoch = 0
        self._new_epoch()

    def _new_epoch(self):
        # the reference never calls set_epoch: every epoch replays the same order
        self.idx = epoch_indices(len(self.ds), self.world, self.rank, self.distributed, self.seed, 0)
        self.pos = 0

    def _next_index(self):
        if self.pos + self.B > len(self.idx):      # drop_last=False in the reference; restart like StopIteration
            if self.pos < len(self.idx):
                sel = self.idx[self.pos:]
                self.pos = len(self.idx)
                return sel
            self.epoch += 1
            self._new_epoch()
        sel = self.idx[self.pos:self.pos + self.B]
        self.pos += self.B
        return sel

    def __iter__(self):
        return self


class DeviceBatcher(_Batcher):
    def __init__(self, ds, batch_size, world, rank, distributed, device, shuffle_seed=0):
        super().__init__(ds, batch_size, world, rank, distributed, shuffle_seed)
        self.table = ds.data.to(device)
        self.device = device
        self._idx_dev = self.idx.to(device)

    def _new_epoch(self):
        super()._new_epoch()
        if hasattr(self, "table"):
            self._idx_dev = self.idx.to(self.device)

    def __next__(self):
        start = self.pos
        sel = self._next_index()
        if len(sel) == self.B and start + self.B == self.pos:
            return self.table.index_select(0, self._idx_dev[start:start + self.B])
        return self.table.index_select(0, sel.to(self.device))


class HostBatcher(_Batcher):
    def __init__(self, ds, batch_size, world, rank, distributed, device, shuffle_seed=0):
        super().__init__(ds, batch_size, world, rank, distributed, shuffle_seed)
        self.device = device
        self.pin = torch.device(device).type == "cuda"

    def __next__(self):
        b = self.ds.data.index_select(0, self._next_index())
        if self.pin:
            b = b.pin_memory()
        return b.to(self.device, non_blocking=True)


def make_batcher(kind, ds, batch_size, world, rank, strategy, device):
    distributed = world > 1 and strategy in ("ddp", "fsdp")
    cls = DeviceBatcher if kind == "device" else HostBatcher
    return cls(ds, batch_size, world, rank, distributed, device, shuffle_seed=0 if distributed else 42)
