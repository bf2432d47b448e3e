"""The hot path on N GPUs, one process per GPU.

Partitioning (``scaling: strong`` -- the panel is fixed, N GPUs share it):

* **Assets**, in whole blocks of the fixed 8-block split, for the factor build, the z-score
  statistics and the Gram partials: pandas' rolling/ewm states carry rounding history from each
  asset's first day, so an exact factor panel needs each asset's whole series on one device (an
  asset shard is exact; a date shard would have to replay every running state from day 0).
* Every sum over assets follows a fixed binary tree whose leaves are the 8 blocks (and, inside a
  block, its 64-asset row-blocks): a rank computes its subtree, the exchange carries subtree
  results, and the results are bit-identical for N = 1, 2, 4, 8.
* **Dates** for the per-date FM regressions (one all_to_all of per-date partials to the date
  owners), the rebalance (an even split, results all-gathered) -- every rank then runs the
  sequential PnL scan.

Inputs are replicated: every rank builds the full input grid (the seeded generator, or its own
copy of the reference frame), so history / close / tmr planes need no exchange.

``Comm`` wraps torch.distributed: RCCL (backend "nccl") on device tensors; with backend "gloo"
tensors are staged through host memory (CPU tests, or several ranks sharing one GPU).
"""
from __future__ import annotations

from .grid import PanelGrid
from .pipeline import EXCHANGE_STAGES, Pipeline, PipelineConfig  # noqa: F401


def block_range(n: int, world: int, rank: int, unit: int = 64):
    """[lo, hi) of ``rank``'s share of ``n`` items split in whole ``unit``-blocks (the last
    block may be short)."""
    nb = (n + unit - 1) // unit
    b0, b1 = nb * rank // world, nb * (rank + 1) // world
    return min(unit * b0, n), min(unit * b1, n)


def even_range(n: int, world: int, rank: int):
    return n * rank // world, n * (rank + 1) // world


class Comm:
    """Collectives of one process group (torch.distributed)."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.host = dist.get_backend(group) == "gloo"

    def _stage(self, t):
        return t.cpu() if self.host else t

    def all_gather(self, t):
        """Equal-shape all-gather -> tensor [world, *t.shape] on t's device."""
        import torch
        src = self._stage(t.contiguous())
        if self.host:
            parts = [torch.empty_like(src) for _ in range(self.world)]
            self.dist.all_gather(parts, src, group=self.group)
            out = torch.stack(parts)
        else:
            # the ranks' tensors concatenated along dim 0 (the output form every backend takes;
            # the stacked form is NCCL-only), then viewed [world, *t.shape]
            flat = src if src.dim() else src.reshape(1)
            out = torch.empty((self.world * flat.shape[0],) + tuple(flat.shape[1:]),
                              dtype=src.dtype, device=src.device)
            self.dist.all_gather_into_tensor(out, flat, group=self.group)
            out = out.view((self.world,) + tuple(src.shape))
        return out.to(t.device)

    def all_gather_packed(self, tensors):
        """Several equal-shape-per-rank tensors of any dtypes in ONE all-gather (their bytes
        concatenated) -> list of [world, *t.shape] tensors."""
        import torch
        flat = [t.contiguous().view(-1).view(torch.uint8) for t in tensors]
        sizes = [f.numel() for f in flat]
        g = self.all_gather(torch.cat(flat))                     # [world, total bytes]
        out, off = [], 0
        for t, n in zip(tensors, sizes):
            # a strided view of the gathered bytes when the part's offset and the row stride are
            # multiples of its element size (no copy of the gathered buffer), else a copy
            es = t.element_size()
            part = g[:, off:off + n]
            if off % es or g.shape[1] % es:
                part = part.contiguous()
            part = part.view(t.dtype)
            out.append(part.view((self.world,) + tuple(t.shape)))
            off += n
        return out

    def all_gather_buffer(self, sb):
        """ONE all-gather of a ``packing.SendBuffer`` -> its parts as [world, *shape] views."""
        from .packing import unpack_gathered
        return unpack_gathered(self.all_gather(sb.buf), sb.layout, self.world)

    def all_to_all(self, inp, in_splits, out_splits):
        """all_to_all_single along dim 0 with explicit split sizes (rows)."""
        import torch
        src = self._stage(inp.contiguous())
        out = torch.empty((sum(out_splits),) + tuple(src.shape[1:]), dtype=src.dtype,
                          device=src.device)
        self.dist.all_to_all_single(out, src, output_split_sizes=list(out_splits),
                                    input_split_sizes=list(in_splits), group=self.group)
        return out.to(inp.device)

    def barrier(self):
        self.dist.barrier(group=self.group)


class EmulatedComm:
    """One rank of a ``world``-rank job in a single process, for measuring what a rank computes
    (``bench.py --emulate-world N``): every collective returns this rank's own contribution in
    every other rank's slot, so the step runs exactly rank ``rank``'s kernels -- its asset shard,
    its date shares -- on its own shapes, with no communication.  The results are not the
    job's results (the other ranks' shares are copies); this is a timing device only."""

    def __init__(self, world: int, rank: int = 0):
        if world < 2 or not 0 <= rank < world:
            raise ValueError("need world >= 2 and 0 <= rank < world")
        self.world, self.rank, self.host = world, rank, False

    def all_gather(self, t):
        return t.contiguous().unsqueeze(0).expand((self.world,) + tuple(t.shape)).contiguous()

    def all_gather_packed(self, tensors):
        return [self.all_gather(t) for t in tensors]

    def all_gather_buffer(self, sb):
        from .packing import unpack_gathered
        return unpack_gathered(self.all_gather(sb.buf), sb.layout, self.world)

    def all_to_all(self, inp, in_splits, out_splits):
        import torch
        off = sum(in_splits[:self.rank])
        own = inp[off:off + in_splits[self.rank]]
        parts = []
        for n in out_splits:                      # every sender's block: this rank's own rows
            reps = -(-n // max(own.shape[0], 1))
            parts.append(own.repeat((reps,) + (1,) * (own.dim() - 1))[:n] if own.shape[0]
                         else torch.zeros((n,) + tuple(inp.shape[1:]), dtype=inp.dtype,
                                          device=inp.device))
        return torch.cat(parts)

    def barrier(self):
        pass


def ShardedPipeline(grid: PanelGrid, comm: Comm, cfg: PipelineConfig | None = None) -> Pipeline:
    """``Pipeline.step()`` on one rank of ``comm.world`` (afm.pipeline.Pipeline with a comm):
    bit-identical to the single-device step for N in {1, 2, 4, 8}."""
    return Pipeline(grid, cfg, comm)


def gather_path_series(local: dict, npaths: int, comm: Comm) -> dict:
    """The per-path series of every rank's path share (``even_range`` of ``npaths``) in ONE
    all-gather (shares padded to the largest) -> the full [npaths][...] series on every rank."""
    import torch
    keys = ("value", "turnover", "long_ret", "short_ret")
    nmax = -(-npaths // comm.world)
    padded = []
    for k in keys:
        t = local[k]
        pad = torch.zeros((nmax,) + tuple(t.shape[1:]), dtype=t.dtype, device=t.device)
        pad[:t.shape[0]] = t
        padded.append(pad)
    got = comm.all_gather_packed(padded)
    out = {}
    for k, g in zip(keys, got):
        parts = []
        for q in range(comm.world):
            lo, hi = even_range(npaths, comm.world, q)
            parts.append(g[q, :hi - lo])
        out[k] = torch.cat(parts)
    return out


def bootstrap_pnl_sharded(reb: dict, pred, dates_idx, paths, comm: Comm, v0=None, rate=1e-4):
    """Config E on N GPUs: the bootstrap paths split evenly over the ranks (each path's value /
    turnover recursion is independent -- no exchange while they run), then one all-gather of the
    PnL series.  ``reb`` / ``pred`` are the (replicated) rebalance outputs of the sharded step."""
    import numpy as np
    from .portfolio import V0, bootstrap_pnl
    paths = np.asarray(paths, dtype=np.int32)
    lo, hi = even_range(len(paths), comm.world, comm.rank)
    local = bootstrap_pnl(reb, pred, dates_idx, paths[lo:hi], V0 if v0 is None else v0, rate)
    return gather_path_series(local, len(paths), comm)
