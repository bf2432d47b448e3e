"""The z-scored Gram kernels at the widest designs the entry points accept (p = 97 .. 106), against
a torch fp64 D^T D of the same rows (D = [1, (x - mu) * (1/sigma), y], the kernels' z).

BASELINE config C names "100 factors": from p = 100 a ring slot ((p + 4) x 66 doubles) no longer
fits three times in LDS, so zgram_kernel runs with two slots, and from p = 99 the border wave
carries 3..12 columns.  Both afm_zpool_f64 (row-block x date-chunk leaves, the pooled Gram of
KKT:582-583 / :605-607) and afm_zgram_f64 (per (date, asset block), the per-date Grams) are run
on a small ragged panel with an asset range that ends inside a row-block.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

T, LDA, A_END = 150, 256, 229       # dates, padded assets, assets present (ends mid row-block)


def _case(p, seed):
    import torch
    rng = np.random.default_rng(seed)
    ncol = p + 3                                         # planes: p features + y + 2 unused
    base = rng.normal(5.0, 10.0, size=(ncol, T, LDA))
    cols = rng.permutation(ncol - 1)[:p].astype(np.int32)
    ycol = int(np.setdiff1d(np.arange(ncol - 1), cols)[0])
    mu = rng.normal(4.0, 3.0, size=(p, LDA))
    rs = 1.0 / rng.uniform(0.5, 20.0, size=(p, LDA))
    zs = np.zeros((p + 1, LDA, 2))
    zs[:p, :, 0], zs[:p, :, 1] = mu, rs
    zs[p, :, 1] = 1.0                                    # identity row: y passes unchanged
    keep = rng.random((T, LDA)) < 0.8
    keep[:, A_END:] = False
    keep[40] = False                                     # an empty date
    words = np.zeros(((T + 63) // 64, LDA), np.uint64)
    for t in range(T):
        words[t // 64] |= keep[t].astype(np.uint64) << np.uint64(t % 64)
    dev = "cuda"
    return dict(base=torch.from_numpy(base).to(dev), cols=torch.from_numpy(cols).to(dev),
                ycol=ycol, zs=torch.from_numpy(zs).to(dev),
                bits=torch.from_numpy(words.view(np.int64)).to(dev), keep=keep, p=p,
                np_base=base, np_cols=cols, mu=mu, rs=rs)


def _ref_gram(c, t0, t1):
    """fp64 D^T D over the kept rows of dates [t0, t1) (numpy, exact products, pairwise sums)."""
    p = c["p"]
    tt, aa = np.nonzero(c["keep"][t0:t1])
    tt = tt + t0
    X = c["np_base"][c["np_cols"]][:, tt, aa]                       # [p][n]
    Z = (X - c["mu"][:, aa]) * c["rs"][:, aa]
    y = c["np_base"][c["ycol"]][tt, aa]
    D = np.concatenate([np.ones((1, len(y))), Z, y[None]], axis=0)   # [p + 2][n]
    return D @ D.T


def _close(got, ref, what):
    scale = np.abs(ref).max()
    err = np.abs(got - ref).max() / scale
    assert err < 1e-12, (what, err)


@pytest.mark.parametrize("p", [97, 99, 100, 103, 106])
def test_zpool_wide_vs_fp64(p):
    """afm_zpool_f64: 4 row-blocks x 5 date chunks of [0, T), then the fixed tree to one Gram."""
    import torch
    from afm import _lib
    L, P, chk = _lib.lib(), _lib.ptr, _lib.check
    c = _case(p, seed=p)
    pe = L.afm_zgram_part_bytes(p) // 8
    nrb, nchunk = LDA // 64, 5
    part = torch.full((nrb * nchunk, pe), float("nan"), dtype=torch.float64, device="cuda")
    G = torch.empty((1, p + 2, p + 2), dtype=torch.float64, device="cuda")
    h = _lib.Context.get(0).bind_stream()
    chk(L.afm_zpool_f64(h, P(c["base"]), T * LDA, LDA, P(c["cols"]), None, p, c["ycol"],
                        P(c["zs"]), p, P(c["bits"]), 0, T, 0, nrb, A_END, nchunk, P(part), 0),
        "zpool")
    chk(L.afm_gram_tree_f64(h, p, P(part), nrb * nchunk, nrb * nchunk, 1, P(G)), "tree")
    torch.cuda.synchronize()
    got = G[0].cpu().numpy()
    ref = _ref_gram(c, 0, T)
    assert got[0, 0] == ref[0, 0]                        # the row count is exact
    _close(got, ref, f"zpool p={p}")
    assert np.array_equal(got, got.T)


@pytest.mark.parametrize("p", [97, 100, 106])
def test_zgram_per_date_wide_vs_fp64(p):
    """afm_zgram_f64 (mode 0): one partial per (date, 128-asset block), merged per date."""
    import torch
    from afm import _lib
    L, P, chk = _lib.lib(), _lib.ptr, _lib.check
    c = _case(p, seed=1000 + p)
    pe = L.afm_zgram_part_bytes(p) // 8
    t0, nt, nblk, blk = 30, 24, 2, 128
    part = torch.full((nt * nblk, pe), float("nan"), dtype=torch.float64, device="cuda")
    G = torch.empty((nt, p + 2, p + 2), dtype=torch.float64, device="cuda")
    h = _lib.Context.get(0).bind_stream()
    chk(L.afm_zgram_f64(h, P(c["base"]), T * LDA, LDA, P(c["cols"]), None, p, c["ycol"],
                        P(c["zs"]), p, P(c["bits"]), t0, nt, nblk, 0, blk, A_END, P(part), 0),
        "zgram")
    chk(L.afm_gram_tree_f64(h, p, P(part), nt * nblk, nblk, 1, P(G)), "tree")
    torch.cuda.synchronize()
    got = G.cpu().numpy()
    for d in range(nt):
        ref = _ref_gram(c, t0 + d, t0 + d + 1)
        if ref[0, 0] == 0:                               # the empty date: an all-zero Gram
            assert (got[d] == 0).all()
            continue
        assert got[d, 0, 0] == ref[0, 0]
        _close(got[d], ref, f"zgram p={p} date {t0 + d}")


def _ref_raw_gram(c, t, a0, a1):
    """fp64 D^T D of the raw FM design D = [1, x, y] over the kept rows of date t, assets
    [a0, a1)."""
    aa = np.nonzero(c["keep"][t, a0:a1])[0] + a0
    X = c["np_base"][c["np_cols"]][:, t, aa]
    y = c["np_base"][c["ycol"]][t, aa]
    D = np.concatenate([np.ones((1, len(aa))), X, y[None]], axis=0)
    return D @ D.T


@pytest.mark.parametrize("p", [30, 17, 5])
def test_fm_raw_per_date_gram_vs_fp64(p):
    """afm_zgram_f64 without z statistics (the FM30 per-date Grams of KKT:630-631), per (date,
    128-asset block) partial, against fp64 numpy; a block past a_end (an all-zero partial), an
    empty date, a ragged block."""
    import torch
    from afm import _lib
    L, P, chk = _lib.lib(), _lib.ptr, _lib.check
    c = _case(p, seed=2000 + p)
    pe = L.afm_zgram_part_bytes(p) // 8
    t0, nt, nblk, blk = 30, 24, 3, 128                   # block 2 lies past a_end = 229
    part = torch.full((nt * nblk, pe), float("nan"), dtype=torch.float64, device="cuda")
    G = torch.empty((nt * nblk, p + 2, p + 2), dtype=torch.float64, device="cuda")
    h = _lib.Context.get(0).bind_stream()
    chk(L.afm_zgram_f64(h, P(c["base"]), T * LDA, LDA, P(c["cols"]), None, p, c["ycol"],
                        None, 0, P(c["bits"]), t0, nt, nblk, 0, blk, A_END, P(part), 0),
        "zgram fm")
    chk(L.afm_gram_tree_f64(h, p, P(part), nt * nblk, 1, 1, P(G)), "tree")
    torch.cuda.synchronize()
    got = G.cpu().numpy().reshape(nt, nblk, p + 2, p + 2)
    for d in range(nt):
        for b in range(nblk):
            a0, a1 = b * blk, min((b + 1) * blk, A_END)
            g = got[d, b]
            if a1 <= a0 or not c["keep"][t0 + d, a0:a1].any():
                assert (g == 0).all(), (d, b)
                continue
            ref = _ref_raw_gram(c, t0 + d, a0, a1)
            assert g[0, 0] == ref[0, 0]                  # the row count is exact
            _close(g, ref, f"fm p={p} date {t0 + d} block {b}")
            assert np.array_equal(g, g.T)
