"""Lasso row (KKT:605-607): the oracle's Gram coordinate descent vs the
scikit-learn fits in tests/golden/lasso_sklearn.npz (CPU), and on the GPU afm_lasso_cd_f64 vs the
oracle on the same pooled moments (bit-exact) and afm.Lasso vs scikit-learn.

Tolerances: scikit-learn runs residual-form coordinate descent with BLAS reductions, the oracle
and the kernel the Gram form with sequential ones, so iterates differ by rounding: coefficients
agree to 1e-9 of max|coef| at tol 1e-12; at the reference's tol 1e-4 both stop on the same duality
gap test, so n_iter agrees and the coefficients agree to 1e-6 of max|coef|."""
import os

import numpy as np
import pytest

CASES = ["ref", "sparse", "positive", "capped"]


def _golden(golden_dir):
    return np.load(os.path.join(golden_dir, "lasso_sklearn.npz"))


def _oracle_fit(X, y, alpha, max_iter, tol, positive):
    import oracle
    n = len(y)
    xm, ym = X.mean(0), y.mean()
    Xc, yc = X - xm, y - ym
    w, gap, tol_y, it = oracle.lasso_gram(Xc.T @ Xc, Xc.T @ yc, yc @ yc, alpha * n,
                                          max_iter=max_iter, tol=tol, positive=positive)
    return w, ym - xm @ w, it, gap / n


@pytest.mark.parametrize("case", CASES)
@pytest.mark.parametrize("tol", [4, 12])
def test_oracle_matches_sklearn(golden_dir, case, tol):
    g = _golden(golden_dir)
    alpha, max_iter, pos = g[f"{case}_params"]
    w, b, it, gap = _oracle_fit(g[f"{case}_X"], g[f"{case}_y"], alpha, int(max_iter),
                                10.0 ** -tol, bool(pos))
    k = f"{case}_tol{tol}"
    ref = g[f"{k}_coef"]
    scale = max(np.abs(ref).max(), 1e-300)
    bar = 1e-9 if tol == 12 else 1e-6
    assert np.abs(w - ref).max() <= bar * scale
    assert abs(b - float(g[f"{k}_intercept"])) <= bar * scale
    assert it == int(g[f"{k}_n_iter"])
    assert np.array_equal(w == 0, ref == 0) or tol == 4


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_kernel_bit_exact_vs_oracle(golden_dir, case):
    import torch
    import oracle
    from afm import _lib
    from afm.regression import SEG_ROWS, pool_moments, xs_gram
    g = _golden(golden_dir)
    X, y = g[f"{case}_X"], g[f"{case}_y"]
    alpha, max_iter, pos = g[f"{case}_params"]
    n, p = X.shape
    Z = torch.from_numpy(np.ascontiguousarray(np.concatenate([X, y[:, None]], 1).T)).cuda()
    nseg = (n + SEG_ROWS - 1) // SEG_ROWS
    gram, shift = xs_gram(Z, n, SEG_ROWS, SEG_ROWS, list(range(p)), p, nseg=nseg, row_limit=n)
    G, _ = pool_moments(gram, shift, p)
    for tol in (1e-4, 1e-12):
        w = torch.empty(p, dtype=torch.float64, device="cuda")
        info = torch.empty(3, dtype=torch.float64, device="cuda")
        h = _lib.Context.get(0).bind_stream()
        _lib.check(_lib.lib().afm_lasso_cd_f64(h, _lib.ptr(G), p, float(alpha) * n, 0.0,
                                               int(max_iter), tol, int(pos), _lib.ptr(w),
                                               _lib.ptr(info)))
        nn, Q, q, yy = oracle.centered_moments(G[0].cpu().numpy())
        wo, gap, tol_y, it = oracle.lasso_gram(Q, q, yy, float(alpha) * nn, max_iter=int(max_iter),
                                               tol=tol, positive=bool(pos))
        assert np.array_equal(w.cpu().numpy(), wo)
        assert info.cpu().numpy().tolist() == [gap, tol_y, float(it)]


@pytest.mark.gpu
@pytest.mark.parametrize("case", CASES)
def test_lasso_dropin_matches_sklearn(golden_dir, case):
    import warnings

    import pandas as pd
    import afm
    g = _golden(golden_dir)
    X, y = g[f"{case}_X"], g[f"{case}_y"]
    alpha, max_iter, pos = g[f"{case}_params"]
    Xdf = pd.DataFrame(X, columns=[f"f{i}" for i in range(X.shape[1])])
    for tol in (4, 12):
        with warnings.catch_warnings():
            warnings.simplefilter("ignore")
            m = afm.Lasso(alpha=float(alpha), max_iter=int(max_iter), tol=10.0 ** -tol,
                          positive=bool(pos)).fit(Xdf, pd.DataFrame({"target": y}))
        k = f"{case}_tol{tol}"
        ref = g[f"{k}_coef"]
        scale = max(np.abs(ref).max(), 1e-300)
        bar = 1e-9 if tol == 12 else 1e-6
        assert m.coef_.shape == ref.shape and np.shape(m.intercept_) == (1,)
        assert np.abs(m.coef_ - ref).max() <= bar * scale
        assert abs(m.intercept_[0] - float(g[f"{k}_intercept"])) <= bar * scale
        assert m.n_iter_ == int(g[f"{k}_n_iter"])
        pred = m.predict(Xdf)
        want = X @ ref + float(g[f"{k}_intercept"])
        assert np.abs(pred - want).max() <= 10 * bar * scale * (1 + np.abs(X).max())
    assert list(m.feature_names_in_) == list(Xdf.columns)


@pytest.mark.gpu
def test_lasso_rejects_nonfinite():
    import afm
    X = np.ones((10, 2))
    X[3, 1] = np.nan
    with pytest.raises(ValueError):
        afm.Lasso(alpha=0.1).fit(X, np.zeros(10))


@pytest.mark.gpu
@pytest.mark.parametrize("p,alpha,pos", [(96, 2e-4, 0), (110, 5e-5, 0), (70, 1e-4, 1)])
def test_kernel_dense_fit_bit_exact_vs_oracle(p, alpha, pos):
    """Dense fits (many coefficients move every sweep, hundreds of sweeps, both column halves):
    the kernel's pipelined coordinate step -- the next movable coordinate's inputs read while the
    current one computes, confirmed by the ballot after its update -- against the oracle's
    sequential descent, bit for bit (signed zeros included)."""
    import torch
    import oracle
    from afm import _lib
    rng = np.random.default_rng(p)
    n = 4000
    F = rng.normal(size=(n, 6))
    X = F @ rng.normal(size=(6, p)) + 0.5 * rng.normal(size=(n, p))   # correlated columns
    beta = np.where(rng.random(p) < 0.4, rng.normal(size=p), 0.0)
    y = X @ beta + rng.normal(size=n)
    Z = np.concatenate([np.ones((n, 1)), X, y[:, None]], 1)
    G = torch.from_numpy(Z.T @ Z).cuda().contiguous()           # raw moments [1, x, y]
    nn, Q, q, yy = oracle.centered_moments(G.cpu().numpy())
    for tol in (1e-4, 1e-10):
        w = torch.empty(p, dtype=torch.float64, device="cuda")
        info = torch.empty(3, dtype=torch.float64, device="cuda")
        h = _lib.Context.get(0).bind_stream()
        _lib.check(_lib.lib().afm_lasso_cd_f64(h, _lib.ptr(G), p, alpha * n, 0.0, 10000, tol, pos,
                                               _lib.ptr(w), _lib.ptr(info)))
        wo, gap, tol_y, it = oracle.lasso_gram(Q, q, yy, alpha * nn, max_iter=10000, tol=tol,
                                               positive=bool(pos))
        assert (wo != 0).sum() >= 10 and it >= 5
        assert w.cpu().numpy().tobytes() == wo.tobytes()
        assert info.cpu().numpy().tolist() == [gap, tol_y, float(it)]


@pytest.mark.gpu
def test_kernel_engine_dense_gram_bit_exact_vs_oracle(golden_dir):
    """The bench's `dense_lasso` fit itself: the engine's pooled Gram of the config-C dense
    variant (tests/golden/lasso_dense_gram.npz, saved by `LASSO_SAVE=<dir> tools/lasso_probe.py`
    from the engine's own pooled moments: 96 features, alpha 2e-6, 1,936 sweeps, 20 nonzero
    coefficients) -- afm_lasso_fit_f64 against the oracle's descent on the same moments, bit for
    bit (signed zeros included), and the fit's coefficients and sweep count as saved."""
    import torch
    import oracle
    from afm import _lib
    d = np.load(os.path.join(golden_dir, "lasso_dense_gram.npz"))
    p, alpha, max_iter, tol = int(d["p"]), float(d["alpha"]), int(d["max_iter"]), float(d["tol"])
    G = torch.from_numpy(d["gram"]).cuda().contiguous()
    S = torch.from_numpy(d["shift"]).cuda().contiguous()
    beta = torch.empty(p + 1, dtype=torch.float64, device="cuda")
    info = torch.empty(3, dtype=torch.float64, device="cuda")
    h = _lib.Context.get(0).bind_stream()
    _lib.check(_lib.lib().afm_lasso_fit_f64(h, _lib.ptr(G), _lib.ptr(S), p, alpha, max_iter, tol,
                                            0, _lib.ptr(beta), _lib.ptr(info)))
    nn, Q, q, yy = oracle.centered_moments(d["gram"][0])
    wo, gap, tol_y, it = oracle.lasso_gram(Q, q, yy, alpha * nn, max_iter=max_iter, tol=tol)
    b = beta.cpu().numpy()
    assert it == 1936 and (wo != 0).sum() == 20
    assert b[1:].tobytes() == wo.tobytes()
    assert info.cpu().numpy().tolist() == [gap, tol_y, float(it)]
    assert b.tobytes() == d["beta"].tobytes()
