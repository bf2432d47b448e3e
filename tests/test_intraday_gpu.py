"""Config D (intraday minute bars): long series through the factor kernel and the asset-group
streaming build (afm/intraday.py) -- bit-exact against the oracle and against one launch."""
import numpy as np
import pytest

from helpers import mismatch_report, same

pytestmark = pytest.mark.gpu


def _oracle_of(grid):
    import oracle
    v = grid.valid[:, :grid.A].cpu().numpy()
    aa, tt = np.nonzero(v.T)
    off = np.r_[0, np.cumsum(v.sum(axis=0))].astype(np.int64)
    c = lambda x: x[:, :grid.A].cpu().numpy()[tt, aa]     # noqa: E731
    fac = oracle.factors_long(off, c(grid.close), c(grid.volume), c(grid.ret1d),
                              c(grid.excess))
    return tt, aa, fac


def test_minute_bar_series_vs_oracle():
    """200,000 bars per asset (longer than config D's 196,560): no state or index wraps."""
    import torch
    import afm
    from afm.intraday import make_panel_device
    torch.cuda.set_device(0)
    g = make_panel_device(6, 200_000, seed=11, hole_frac=0.01, listing_frac=0.05)
    out, nanfree = afm.factor_panel(g)
    tt, aa, ref = _oracle_of(g)
    got = out[:, torch.from_numpy(tt).cuda(), torch.from_numpy(aa).cuda()].T.cpu().numpy()
    assert same(got, ref), mismatch_report(got, ref, afm.FACTOR_NAMES)
    # nanfree = present and no NaN among the 96 factors
    bits = afm.unpack_bits(nanfree, g.T)[:, :g.A].cpu().numpy()
    want = np.zeros_like(bits)
    want[tt, aa] = ~np.isnan(ref[:, :96]).any(axis=1)
    assert np.array_equal(bits, want)


@pytest.mark.parametrize("bpg", [1, 2, 5])
def test_asset_groups_identical_to_one_launch(bpg):
    import torch
    import afm
    from afm.intraday import factor_panel_groups, make_panel_device
    torch.cuda.set_device(0)
    g = make_panel_device(300, 2500, seed=5, hole_frac=0.01)
    full, nf_full = afm.factor_panel(g)
    vb = afm.unpack_bits(g.vbits, g.T)
    seen = []

    def consume(a0, a1, out, nanfree):
        w = a1 - a0
        m = vb[:, a0:a1]
        a, b = out[:, :, :w][:, m], full[:, :, a0:a1][:, m]
        assert torch.equal(torch.isnan(a), torch.isnan(b))
        assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b))
        assert torch.equal(nanfree[:, :w], nf_full[:, a0:a1])
        seen.append((a0, a1))

    n = factor_panel_groups(g, consume, blocks_per_group=bpg)
    nblk = (g.A + 63) // 64
    assert n == (nblk + bpg - 1) // bpg
    assert seen[0][0] == 0 and seen[-1][1] == g.A
    assert all(x[1] == y[0] for x, y in zip(seen, seen[1:]))


def test_group_sizing():
    import torch
    from afm.intraday import group_blocks, make_panel_device
    torch.cuda.set_device(0)
    g = make_panel_device(3000, 640, seed=1)
    per_blk = 102 * 8 * 640 * 64
    assert group_blocks(g, budget_bytes=10**15) == 47                  # everything in one
    b = group_blocks(g, budget_bytes=21 * per_blk + 2 * 8 * 10 * 64 * 21)
    assert b <= 21 and ((47 + b - 1) // b) == 3 and b == 16            # 16, 16, 15


@pytest.mark.parametrize("types,step", [(15, 64), (5, 320), (3, 1024), (3, 704), (110, 64),
                                        (106, 320), (103, 704), (206, 64), (206, 704)])
def test_time_slabs_identical_to_one_launch(monkeypatch, types, step):
    """Config D's default build: ALL assets over consecutive time slabs, every recurrence state
    and observation ring carried across slab boundaries in the state buffer -- the concatenated
    slabs (98 planes incl. the labels, nanfree bits) equal one launch bit for bit, for every
    workgroup split of the job sets (3 = the paired 12-wave launch; 1xx = the small-grid
    partition, whose loaders also carry the return / volume-change rings)."""
    import torch
    import afm
    from afm.intraday import factor_panel_slabs, make_panel_device
    torch.cuda.set_device(0)
    from afm import _lib
    g = make_panel_device(300, 2500, seed=9, hole_frac=0.01)
    opts = _lib.options(factor_split=types)
    opts.__enter__()
    full, nf_full = afm.factor_panel(g)
    vb = afm.unpack_bits(g.vbits, g.T)
    seen = []

    def consume(t0, t1, out, nanfree):
        m = vb[t0:t1]
        a, b = out[:, m], full[:, t0:t1][:, m]
        assert torch.equal(torch.isnan(a), torch.isnan(b)), (t0, t1)
        assert torch.equal(torch.nan_to_num(a), torch.nan_to_num(b)), (t0, t1)
        w0, w1 = t0 // 64, (t1 + 63) // 64
        assert torch.equal(nanfree, nf_full[w0:w1]), (t0, t1)
        seen.append((t0, t1))

    try:
        n = factor_panel_slabs(g, consume, bars_per_slab=step)
    finally:
        opts.__exit__(None, None, None)
    assert n == (g.T + step - 1) // step and seen[-1][1] == g.T


def test_config_d_full_size_slabs_vs_oracle():
    """BASELINE config D at full size: 3,000 assets x 196,560 one-minute bars (2 years x 252 days
    x 390 bars, 5.6e8 present asset-bars) through the default time-slab build (factor_panel_slabs,
    output buffer sized to the free HBM).  The consumer keeps 3 sampled assets' 98 columns and
    nanfree bits from every slab; they are compared with the oracle's pandas-exact restatement
    of each asset's whole series (bit-exact), and every slab's nanfree words must be a subset of
    the presence words."""
    import torch
    import afm
    import oracle
    from afm.intraday import factor_panel_slabs, make_panel_device
    torch.cuda.set_device(0)
    A, T = 3000, 2 * 252 * 390
    g = make_panel_device(A, T, seed=2024)
    picks = [0, 1499, 2999]                            # first, middle, last (partial block) asset
    cols = {a: [] for a in picks}
    nfs = {a: [] for a in picks}
    nslab = []

    def consume(t0, t1, out, nanfree):
        nw = (t1 - t0 + 63) // 64
        assert torch.equal(nanfree & ~g.vbits[t0 // 64:t0 // 64 + nw], torch.zeros_like(nanfree))
        for a in picks:
            cols[a].append(out[:, :, a].cpu().numpy())                     # [98][t1 - t0]
            nfs[a].append(afm.unpack_bits(nanfree[:, a:a + 1].contiguous(), t1 - t0)[:, 0].cpu().numpy())
        nslab.append((t0, t1))

    n = factor_panel_slabs(g, consume)
    assert nslab[0][0] == 0 and nslab[-1][1] == T and n == len(nslab)
    vb = afm.unpack_bits(g.vbits, T)
    for a in picks:
        v = vb[:, a].cpu().numpy()
        tt = np.flatnonzero(v)
        x = lambda t: t[:, a].cpu().numpy()[tt]                              # noqa: E731
        ref = oracle.factors_long(np.array([0, len(tt)], np.int64), x(g.close), x(g.volume),
                                  x(g.ret1d), x(g.excess))
        got = np.concatenate(cols[a], axis=1)[:, tt].T
        assert same(got, ref), (a, mismatch_report(got, ref, afm.FACTOR_NAMES))
        nf = np.concatenate(nfs[a])
        want = np.zeros(T, bool)
        want[tt] = ~np.isnan(ref[:, :96]).any(axis=1)
        assert np.array_equal(nf, want), a


def test_slab_default_size_unaligned_series():
    """slab_bars' default on a series that fits one slab and is not a multiple of 64 bars (the
    round-2 advisor case): one slab, equal to one launch."""
    import torch
    import afm
    from afm.intraday import factor_panel_slabs, make_panel_device, slab_bars
    torch.cuda.set_device(0)
    g = make_panel_device(300, 2500, seed=3, hole_frac=0.01)
    assert slab_bars(g) % 64 == 0 and slab_bars(g) >= g.T
    full, nf_full = afm.factor_panel(g)
    vb = afm.unpack_bits(g.vbits, g.T)
    got = []

    def consume(t0, t1, out, nanfree):
        m = vb[t0:t1]
        assert torch.equal(out[:, m].nan_to_num(7.0), full[:, t0:t1][:, m].nan_to_num(7.0))
        assert torch.equal(nanfree, nf_full)
        got.append((t0, t1))

    assert factor_panel_slabs(g, consume) == 1 and got == [(0, g.T)]


def test_slab_split_change_rejected():
    """The carried slab state is laid out per workgroup split ([block][split][wave]): a series
    whose factor_split changes between slabs is rejected before any kernel runs."""
    import torch
    from afm import _lib
    from afm.intraday import factor_panel_slabs, make_panel_device
    torch.cuda.set_device(0)
    g = make_panel_device(130, 300, seed=3)
    ctx = _lib.Context.get()
    before = ctx.get_option("factor_split")
    calls = []

    def consume(t0, t1, out, nanfree):
        calls.append(t0)
        ctx.set_option("factor_split", 5 if before != 5 else 15)

    try:
        with pytest.raises(_lib.AfmError, match="factor_split changed"):
            factor_panel_slabs(g, consume, bars_per_slab=128)
    finally:
        ctx.set_option("factor_split", before)
    assert calls == [0]
