"""Intraday factor panels (BASELINE config D: 3,000 assets x 2 years of 1-minute bars).

The factor build of ``No-talib.py:1-93`` is positional per asset: windows count observations,
not calendar time (``NT:5-6``), so a minute-bar panel runs through the same kernel as a daily
one -- the grid's date axis simply holds bars.  What changes is size.  At 3,000 assets x
196,560 bars the 98 output planes take 98 x 8 x 196,560 x 3,008 B = 463 GB, more than one
MI355X's 288 GB of HBM, and every recurrence is sequential over the whole 196,560-bar series
(pandas' Kahan / Welford states carry their rounding history).

So the build streams: ``factor_panel_slabs`` (the default) runs ALL assets over one TIME SLAB
of bars at a time (``afm_factors_slab_f64``), carrying every recurrence state and observation
ring from slab to slab in a device buffer, into one reused output buffer sized to the free HBM
-- all 47 blocks of config D work at once, where asset groups would leave most CUs idle on a
sequential 196,560-step scan.  ``factor_panel_groups`` streams asset groups instead (assets are
independent, so each group of 64-asset blocks is an exact sub-panel).  Both hand each finished
piece to a consumer callback and are bit-identical to a single launch over the whole panel
(tests/test_intraday_gpu.py).

``make_panel_device`` is the §8(d) generator restated in torch on the device (same
distributions, torch's RNG stream), because a 5.9e8-cell panel is slow to draw with numpy on
the host and to upload.
"""
from __future__ import annotations

import numpy as np

from .factors import N_FACTORS, factor_panel
from .grid import PanelGrid, pack_bits
from .synthetic import LANES, round_up


def make_panel_device(n_assets: int, n_bars: int, seed: int = 2023, *, hole_frac: float = 0.002,
                      listing_frac: float = 0.1, device=None) -> PanelGrid:
    """Synthetic panel generated in HBM: log-price walk (mu 3e-4, sigma
    0.02, start 50), volume round(lognormal(13, 0.5)), listing offsets in [0, T*listing_frac),
    ``hole_frac`` missing cells, ``excess_ret1d`` = ret1d minus the per-bar mean over present
    rows with ret1d <= 1 (KKT:154-161).  Columns past ``n_assets`` are NaN / absent."""
    import torch
    dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
    T, A = int(n_bars), int(n_assets)
    lda = round_up(max(A, 1))
    g = torch.Generator(device=dev)
    g.manual_seed(seed)
    f64 = torch.float64

    close = torch.full((T, lda), float("nan"), dtype=f64, device=dev)
    ret1d = torch.full((T, lda), float("nan"), dtype=f64, device=dev)
    volume = torch.full((T, lda), float("nan"), dtype=f64, device=dev)
    # the walk in slabs of bars (keeps the temporaries small): logp carries across slabs
    carry = torch.full((1, A), float(np.log(50.0)), dtype=f64, device=dev)
    slab = max(1, (1 << 27) // max(A, 1))
    for t0 in range(0, T, slab):
        t1 = min(T, t0 + slab)
        eps = torch.randn((t1 - t0, A), generator=g, dtype=f64, device=dev) * 0.02 + 3e-4
        logp = torch.cumsum(eps, dim=0) + carry
        prev = torch.cat([carry, logp[:-1]], dim=0)
        carry = logp[-1:].clone()
        px = torch.exp(logp)
        close[t0:t1, :A] = px
        ret1d[t0:t1, :A] = px / torch.exp(prev) - 1.0
        volume[t0:t1, :A] = torch.round(torch.exp(
            torch.randn((t1 - t0, A), generator=g, dtype=f64, device=dev) * 0.5 + 13.0))
        del eps, logp, prev, px

    listing = torch.randint(0, max(1, int(T * listing_frac)), (A,), generator=g, device=dev)
    valid = torch.zeros((T, lda), dtype=torch.bool, device=dev)
    excess = torch.full((T, lda), float("nan"), dtype=f64, device=dev)
    for t0 in range(0, T, slab):
        t1 = min(T, t0 + slab)
        tt = torch.arange(t0, t1, device=dev).view(-1, 1)
        v = (tt >= listing.view(1, -1)) & ~(
            torch.rand((t1 - t0, A), generator=g, device=dev) < hole_frac)
        valid[t0:t1, :A] = v
        r = ret1d[t0:t1, :A]
        m = v & (r <= 1.0)
        cnt = m.sum(dim=1, keepdim=True).to(f64)
        s = torch.where(m, r, torch.zeros_like(r)).sum(dim=1, keepdim=True)
        mean = torch.where(cnt > 0, s / cnt.clamp(min=1), torch.zeros_like(s))
        excess[t0:t1, :A] = r - mean
    start = np.datetime64("2000-01-03T09:30", "m")
    dates = (start + np.arange(T).astype("timedelta64[m]")).astype("datetime64[ns]")
    ids = (1000 + 7 * np.arange(A)).astype(np.int64)
    return PanelGrid(dates=dates, ids=ids, close=close, volume=volume, ret1d=ret1d,
                     excess=excess, valid=valid, vbits=pack_bits(valid))


def group_blocks(grid: PanelGrid, budget_bytes: int | None = None) -> int:
    """64-asset blocks per group: the most whose output planes (98 x T x 64 x 8 B per block) plus
    the group's input copies fit in ``budget_bytes`` (default: 85% of the free HBM), balanced so
    the groups have near-equal block counts."""
    import torch
    T = grid.T
    nblk = (grid.A + LANES - 1) // LANES
    if budget_bytes is None:
        free, _ = torch.cuda.mem_get_info(grid.device)
        budget_bytes = int(free * 0.85)
    per_blk = (N_FACTORS + 4) * 8 * T * LANES + 2 * 8 * ((T + 63) // 64) * LANES
    cap = max(1, min(nblk, budget_bytes // per_blk))
    n_groups = (nblk + cap - 1) // cap
    return (nblk + n_groups - 1) // n_groups


def _sub_grid(grid: PanelGrid, a0: int, a1: int) -> PanelGrid:
    """Assets [a0, a1) of a resident grid as a contiguous grid (a0 a multiple of 64)."""
    c1 = round_up(a1 - a0) + a0
    sl = slice(a0, c1)

    def cut(x):
        return x[:, sl].contiguous()
    return PanelGrid(dates=grid.dates, ids=grid.ids[a0:a1], close=cut(grid.close),
                     volume=cut(grid.volume), ret1d=cut(grid.ret1d), excess=cut(grid.excess),
                     valid=grid.valid[:, sl], vbits=cut(grid.vbits))


def factor_panel_groups(grid: PanelGrid, consumer, blocks_per_group: int | None = None):
    """Build the 98-column factor panel of ``grid`` one asset group at a time.

    ``consumer(a0, a1, out, nanfree)`` receives each group: assets ``[a0, a1)`` of ``grid``,
    ``out`` float64 ``[98][T][ldg]`` (column j of the group = asset a0 + j; cells of absent or
    padding assets hold stale values -- consult ``nanfree``), ``nanfree`` int64
    ``[ceil(T/64)][ldg]`` presence-and-no-NaN bits.  The buffers are reused by the next group,
    so the consumer must finish with them (on the current stream) before returning.  Returns
    the number of groups."""
    import torch
    if blocks_per_group is None:
        blocks_per_group = group_blocks(grid)
    ga = int(blocks_per_group) * LANES
    if ga <= 0:
        raise ValueError("blocks_per_group must be positive")
    T = grid.T
    A = grid.A
    ldg = min(ga, round_up(A))
    out = torch.empty((N_FACTORS, T, ldg), dtype=torch.float64, device=grid.device)
    nanfree = torch.empty(((T + 63) // 64, ldg), dtype=torch.int64, device=grid.device)
    n = 0
    for a0 in range(0, A, ga):
        a1 = min(A, a0 + ga)
        sub = _sub_grid(grid, a0, a1)
        w = sub.lda
        o = out if w == ldg else out.view(-1)[: N_FACTORS * T * w].view(N_FACTORS, T, w)
        nf = nanfree if w == ldg else nanfree.view(-1)[: nanfree.shape[0] * w].view(-1, w)
        factor_panel(sub, out=o, nanfree=nf)
        consumer(a0, a1, o, nf)
        del sub
        n += 1
    return n


def slab_bars(grid: PanelGrid, budget_bytes: int | None = None) -> int:
    """Bars per time slab: the most (a multiple of 64) whose output planes and mask words fit in
    ``budget_bytes`` (default: 85% of the free HBM), balanced so the slabs have near-equal
    lengths.  Always a multiple of 64 (slab starts must be word-aligned); it may exceed T when
    one slab holds the whole series -- factor_panel_slabs clamps the last slab to T."""
    import torch
    T, lda = grid.T, grid.lda
    if budget_bytes is None:
        free, _ = torch.cuda.mem_get_info(grid.device)
        budget_bytes = int(free * 0.85)
    per_bar = N_FACTORS * 8 * lda + 2 * 8 * lda // 64 + 16
    cap = max(64, (budget_bytes // per_bar) // 64 * 64)
    n = (T + cap - 1) // cap
    return ((T + n - 1) // n + 63) // 64 * 64


def factor_panel_slabs(grid: PanelGrid, consumer, bars_per_slab: int | None = None):
    """Build the 98-column factor panel of ``grid`` one time slab at a time, all assets at once.

    ``consumer(t0, t1, out, nanfree)`` receives each slab: bars ``[t0, t1)``, ``out`` float64
    ``[98][t1 - t0][lda]`` (absent cells stale -- consult ``nanfree``), ``nanfree`` int64
    ``[ceil((t1 - t0)/64)][lda]``.  The buffers are reused by the next slab, so the consumer
    must finish with them (on the current stream) before returning.  Returns the number of
    slabs."""
    import torch
    from . import _lib
    T, lda = grid.T, grid.lda
    step = int(bars_per_slab) if bars_per_slab is not None else slab_bars(grid)
    if step <= 0 or step % 64:
        raise ValueError("bars_per_slab must be a positive multiple of 64")
    ctx = _lib.Context.get(grid.device.index)
    L, P = _lib.lib(), _lib.ptr
    h = ctx.bind_stream()
    nbytes = int(L.afm_factors_state_bytes(h, grid.A))
    if nbytes < 0:
        raise RuntimeError("afm_factors_state_bytes failed")
    state = torch.empty(max(nbytes // 8, 1), dtype=torch.float64, device=grid.device)
    out = torch.empty((N_FACTORS, min(step, T), lda), dtype=torch.float64, device=grid.device)
    nanfree = torch.empty(((min(step, T) + 63) // 64, lda), dtype=torch.int64, device=grid.device)
    n = 0
    for t0 in range(0, T, step):
        t1 = min(T, t0 + step)
        m = t1 - t0
        o = out if m == out.shape[1] else out.view(-1)[: N_FACTORS * m * lda].view(N_FACTORS, m, lda)
        nw = (m + 63) // 64
        nf = nanfree if nw == nanfree.shape[0] else nanfree[:nw]
        _lib.check(L.afm_factors_slab_f64(ctx.bind_stream(), T, grid.A, lda, t0, t1,
                                          P(grid.close), P(grid.volume), P(grid.ret1d),
                                          P(grid.excess), P(grid.vbits), P(o), P(nf), None,
                                          P(state)), "afm_factors_slab_f64")
        consumer(t0, t1, o, nf)
        n += 1
    return n
