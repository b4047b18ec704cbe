"""Flat-buffer layout planning for the parallelism engines.

Every engine stores parameters and gradients in a few large contiguous buffers instead of one
tensor per parameter (the reference leaves that to torch DDP's Reducer buckets, FSDP's
FlatParameter and DeepSpeed's contiguous_gradients, train_harness.py:207-275):

* parameters are views into the flat buffer (``param.data = flat[off:off+n].view(shape)``), so
  GEMMs read them in place and the optimizer writes them in place;
* gradients are views into a flat gradient buffer written directly by the backward GEMMs;
* a *bucket* is a contiguous byte range of whole units that is reduced by ONE collective call
  (all-reduce, reduce-scatter or all-gather) — no pack/unpack copies;
* with sharding, every bucket is padded to a multiple of ``world_size * align`` so it splits into
  equal per-rank chunks; a rank's *owner space* is the concatenation of its chunks and is where the
  fp32 master weights / Adam moments / gradient accumulators live.

Offsets are aligned to ``align`` elements (default 128 = 256 B for bf16) so every parameter view
and every rank chunk is 16-byte aligned for the vectorised kernels and hipBLASLt.
"""
from dataclasses import dataclass, field
from typing import Dict, List, Sequence, Tuple

from .runtime import Unit

ALIGN = 128


def round_up(x: int, m: int) -> int:
    return (x + m - 1) // m * m


@dataclass
class ParamSlot:
    unit: Unit
    index: int          # parameter index inside the unit
    offset: int         # element offset in the flat buffer
    numel: int
    shape: tuple


@dataclass
class Bucket:
    index: int
    start: int          # element range [start, end) of the flat buffer
    end: int
    units: List[Unit] = field(default_factory=list)
    chunk: int = 0      # per-rank chunk size (end - start) // world_size
    owner_start: int = 0  # offset of this rank's chunk in the owner space

    @property
    def numel(self) -> int:
        return self.end - self.start


@dataclass
class FlatLayout:
    slots: Dict[Tuple[int, int], ParamSlot]   # (id(unit), index) -> slot
    buckets: List[Bucket]
    unit_bucket: Dict[int, int]               # id(unit) -> bucket index
    total: int
    world_size: int

    def slot(self, unit: Unit, i: int) -> ParamSlot:
        return self.slots[(id(unit), i)]

    @property
    def owner_numel(self) -> int:
        return sum(b.chunk for b in self.buckets)


def plan_layout(units: Sequence[Unit], world_size: int = 1, bucket_elems: int = 0,
                align: int = ALIGN, shard: bool = False, param_filter=None,
                solo_tail: int = 0, bucket_max: int = 0, solo_head: int = 0,
                early_elems: int = 0, early_count: int = 0) -> FlatLayout:
    """Lay ``units`` (already in the desired memory order) out in one flat buffer.

    ``bucket_elems``: close a bucket once it holds at least this many elements (0 = one bucket per
    unit).  ``shard``: pad each bucket to ``world_size * align`` for equal reduce-scatter chunks.
    ``param_filter(unit, i) -> bool`` restricts which parameters are placed (ZeRO-3 persistence).
    ``solo_tail``: the last ``solo_tail`` units get a bucket each.  In backward order these are the
    units that finish last (block 0, the tied embedding): their collectives cannot overlap any
    compute, so keeping them out of a large shared bucket shortens the exposed communication tail
    (a 64 MiB bucket of blocks 2..0 + the embedding would start only after the embedding).
    ``solo_head``: the first ``solo_head`` units get a bucket each (in backward order the LM head:
    its collective starts right after the first backward op, and the repeated blocks behind it then
    fill their buckets in whole groups).
    ``early_elems`` / ``early_count``: the first ``early_count`` buckets after the solo head ones close at
    ``early_elems`` instead of ``bucket_elems`` (larger buckets early in the backward -- fewer collectives
    while there is compute to hide them -- and the usual size at its end, which is the start of the
    next forward's parameter all-gathers).
    ``bucket_max``: a hard upper bound (DeepSpeed's ``reduce_bucket_size`` / ``allgather_bucket_size``
    semantics): a unit that would push the open bucket past it starts a new bucket.  Units are never
    split, so a unit larger than the bound forms a bucket of its own.
    """
    slots: Dict[Tuple[int, int], ParamSlot] = {}
    buckets: List[Bucket] = []
    unit_bucket: Dict[int, int] = {}
    off = 0
    cur = None
    pad_to = world_size * align if shard else align
    seen = set()

    def close(b):
        b.end = round_up(b.end, pad_to)
        b.chunk = (b.end - b.start) // world_size if shard else 0
        return b.end

    tail_from = len(units) - max(0, int(solo_tail))
    if early_count > 0 and early_elems > 0:
        # an early bucket only where at least one usual-size bucket of the repeated units stays behind
        # it (the last bucket of the backward, the first all-gather of the next forward)
        regular = sum(u.numel for ui, u in enumerate(units) if max(0, int(solo_head)) <= ui < tail_from)
        if regular < early_count * early_elems + bucket_elems:
            early_count = 0
    def unit_end(u, start):
        """End offset of ``u``'s parameters if placed from ``start`` (same rules as below)."""
        e = start
        for i, p in enumerate(u.params):
            if (param_filter is not None and not param_filter(u, i)) or id(p) in seen:
                continue
            e = round_up(e, align) + p.numel()
        return e

    for ui, u in enumerate(units):
        if ui >= tail_from and cur is not None:
            off = close(cur)
            cur = None
        if bucket_max > 0 and cur is not None and cur.end > cur.start \
                and unit_end(u, cur.end) - cur.start > bucket_max:
            off = close(cur)
            cur = None
        placed = False
        for i, p in enumerate(u.params):
            if param_filter is not None and not param_filter(u, i):
                continue
            if id(p) in seen:          # tied parameter already placed through another unit
                continue
            seen.add(id(p))
            if cur is None:
                cur = Bucket(len(buckets), off, off)
                buckets.append(cur)
            off = round_up(off, align)
            slots[(id(u), i)] = ParamSlot(u, i, off, p.numel(), tuple(p.shape))
            off += p.numel()
            cur.end = off
            placed = True
        if placed:
            cur.units.append(u)
            unit_bucket[id(u)] = cur.index
            # buckets already closed after the solo head ones (the current one is the last in the list)
            n_early = len(buckets) - 1 - min(len(buckets) - 1, max(0, int(solo_head)))
            limit = early_elems if (early_count > 0 and early_elems > 0 and n_early < early_count
                                    and ui >= solo_head) else bucket_elems
            if bucket_elems <= 0 or cur.end - cur.start >= limit or ui >= tail_from or ui < solo_head:
                off = close(cur)
                cur = None
    if cur is not None:
        off = close(cur)
    owner = 0
    for b in buckets:
        b.owner_start = owner
        owner += b.chunk
    return FlatLayout(slots, buckets, unit_bucket, off, world_size)


def owner_segments(layout: FlatLayout, rank: int):
    """(owner_start, length, flat_start) of this rank's chunk of every bucket."""
    return [(b.owner_start, b.chunk, b.start + rank * b.chunk) for b in layout.buckets if b.chunk > 0]
