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


@pytest.mark.parametrize("types,step", [(15, 64), (5, 320), (3, 1024), (3, 704)])
def test_time_slabs_identical_to_one_launch(monkeypatch, types, step):
    """Config D's default build: ALL assets over consecutive time slabs, every recurrence state
    and observation ring carried across slab boundaries in the state buffer -- the concatenated
    slabs (98 planes incl. the labels, nanfree bits) equal one launch bit for bit, for every
    workgroup split of the job sets (3 = the paired 12-wave launch)."""
    import torch
    import afm
    from afm.intraday import factor_panel_slabs, make_panel_device
    torch.cuda.set_device(0)
    monkeypatch.setenv("AFM_FP_TYPES", str(types))
    g = make_panel_device(300, 2500, seed=9, hole_frac=0.01)
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

    n = factor_panel_slabs(g, consume, bars_per_slab=step)
    assert n == (g.T + step - 1) // step and seen[-1][1] == g.T
