"""Cross-sectional / pooled OLS.

* ``LinearRegression`` -- drop-in for the scikit-learn estimator as the reference uses it
  (``KKT Yuliang Jiang.py:582-598``: ``fit(X_df, y_df)``, ``intercept_``, ``coef_``,
  ``predict``).  The Gram of [1, X, y] is built on fp64 MFMA in row segments, the segments are
  combined exactly (Chan), the centered normal equations are solved by a scaled Cholesky.
* ``cross_sectional_ols`` -- the north-star per-date regression (Fama-MacBeth): one Gram per
  date straight from the factor planes, batched solves, FM mean / t-statistics.

All arithmetic runs in csrc/xsreg.hip; torch only holds device buffers.
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .factors import COL, N_FACTORS, TARGET

SEG_ROWS = 4096          # rows per Gram segment in long mode (one workgroup each)
DEFAULT_TOL = 1e-10      # relative pivot threshold of the scaled Cholesky


def _dev():
    import torch
    return torch.device("cuda", torch.cuda.current_device())


def xs_gram(base, col_stride: int, seg_stride: int, seg_rows: int, cols, ycol: int, *,
            bits=None, seg0: int = 0, nseg: int, row_limit: int = -1):
    """Raw binding of afm_xs_gram_f64 -> (gram [nseg][p+2][p+2], shift [nseg][p+2])."""
    import torch
    dev = base.device
    cols_t = torch.as_tensor(np.asarray(cols, dtype=np.int32), device=dev)
    p = int(cols_t.numel())
    gram = torch.empty((nseg, p + 2, p + 2), dtype=torch.float64, device=dev)
    shift = torch.empty((nseg, p + 2), dtype=torch.float64, device=dev)
    ctx = _lib.Context.get(dev.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_xs_gram_f64(
        ctx.bind_stream(), P(base), col_stride, seg_stride, seg_rows, row_limit, P(cols_t), p,
        int(ycol), P(bits) if bits is not None else None, seg0, nseg, P(gram), P(shift)),
        "afm_xs_gram_f64")
    return gram, shift


def ols_solve(gram, shift, p: int, tol: float = DEFAULT_TOL):
    """-> (beta [nseg][p+1] (intercept first), nobs [nseg], rank [nseg])."""
    import torch
    nseg = gram.shape[0]
    dev = gram.device
    beta = torch.empty((nseg, p + 1), dtype=torch.float64, device=dev)
    nobs = torch.empty(nseg, dtype=torch.float64, device=dev)
    rank = torch.empty(nseg, dtype=torch.int32, device=dev)
    ctx = _lib.Context.get(dev.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_ols_solve_f64(ctx.bind_stream(), P(gram), P(shift), p, nseg, tol,
                                            P(beta), P(nobs), P(rank)), "afm_ols_solve_f64")
    return beta, nobs, rank


def pool_moments(gram, shift, p: int):
    """Exact combination of per-segment moments -> (gram [1][p+2][p+2], shift [1][p+2])."""
    import torch
    dev = gram.device
    g = torch.empty((1, p + 2, p + 2), dtype=torch.float64, device=dev)
    s = torch.empty((1, p + 2), dtype=torch.float64, device=dev)
    ctx = _lib.Context.get(dev.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_pool_moments_f64(ctx.bind_stream(), P(gram.contiguous()),
                                               P(shift.contiguous()), p, gram.shape[0], P(g),
                                               P(s)), "afm_pool_moments_f64")
    return g, s


def fama_macbeth(beta, rank):
    """mean_t beta_t and t-statistics over dates with a solved regression."""
    import torch
    k = beta.shape[1]
    m = torch.empty(k, dtype=torch.float64, device=beta.device)
    t = torch.empty(k, dtype=torch.float64, device=beta.device)
    ctx = _lib.Context.get(beta.device.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_fama_macbeth_f64(ctx.bind_stream(), P(beta), P(rank),
                                               beta.shape[0], k, P(m), P(t)),
               "afm_fama_macbeth_f64")
    return m, t


def predict_grid(planes, lda: int, cols, beta, bits, t0: int, nt: int, per_date: bool = False,
                 out=None, ycheck: int = -1):
    """pred[t][a] = beta0 + sum_j beta_j x_j for grid rows with a mask bit (NaN elsewhere)."""
    import torch
    dev = planes.device
    T = planes.shape[1]
    cols_t = torch.as_tensor(np.asarray(cols, dtype=np.int32), device=dev)
    if out is None:
        out = torch.full((T, lda), float("nan"), dtype=torch.float64, device=dev)
    ctx = _lib.Context.get(dev.index)
    P = _lib.ptr
    stride = beta.shape[-1] if per_date else 0
    _lib.check(_lib.lib().afm_predict_f64(ctx.bind_stream(), P(planes), T * lda, lda, t0, nt,
                                          P(cols_t), int(cols_t.numel()), P(beta.contiguous()),
                                          stride, P(bits), int(ycheck), P(out)),
               "afm_predict_f64")
    return out


def cross_sectional_ols(planes, nanfree, lda: int, cols, ycol: int = TARGET, t0: int = 0,
                        nt: int | None = None, A: int | None = None, tol: float = DEFAULT_TOL):
    """Per-date OLS of ``ycol`` on ``cols`` (plane indices of the factor panel) over the rows
    that survive dropna (``nanfree`` bits and finite values).  Returns a dict with the per-date
    ``gram``/``shift`` moments, ``beta`` [nt][p+1], ``nobs``, ``rank``, and FM ``fm_mean``,
    ``fm_t``."""
    T = planes.shape[1]
    nt = T - t0 if nt is None else nt
    A = lda if A is None else A
    p = len(cols)
    gram, shift = xs_gram(planes, T * lda, lda, A, cols, ycol, bits=nanfree, seg0=t0, nseg=nt)
    beta, nobs, rank = ols_solve(gram, shift, p, tol)
    m, t = fama_macbeth(beta, rank)
    return {"gram": gram, "shift": shift, "beta": beta, "nobs": nobs, "rank": rank,
            "fm_mean": m, "fm_t": t}


class LinearRegression:
    """Drop-in for ``sklearn.linear_model.LinearRegression`` (fit_intercept=True) as used by the
    reference (KKT:582-598).  Accepts DataFrames / arrays on the host or torch CUDA tensors."""

    def __init__(self, fit_intercept: bool = True, tol: float = 1e-14, refine: int = 8):
        if not fit_intercept:
            raise NotImplementedError("only fit_intercept=True (the reference's usage)")
        self.fit_intercept = True
        self.tol = tol
        self.refine = refine

    @staticmethod
    def _as_columns(X):
        """-> (device [p][n] float64 column-major matrix, n, p, feature names or None)."""
        import torch
        names = None
        if hasattr(X, "columns"):
            names = np.asarray([str(c) for c in X.columns], dtype=object)
            X = X.to_numpy(dtype=np.float64)
        if isinstance(X, torch.Tensor):
            Xt = X.to(device=_dev(), dtype=torch.float64)
        else:
            Xt = torch.from_numpy(np.ascontiguousarray(np.asarray(X, dtype=np.float64))).to(_dev())
        if Xt.ndim == 1:
            Xt = Xt.view(-1, 1)
        n, p = Xt.shape
        return Xt.T.contiguous(), n, p, names

    def fit(self, X, y):
        import torch
        Xc, n, p, names = self._as_columns(X)
        yv = y.to_numpy(dtype=np.float64) if hasattr(y, "to_numpy") else y
        y2d = (getattr(yv, "ndim", 1) == 2)
        yt = torch.as_tensor(np.asarray(yv, dtype=np.float64) if not isinstance(yv, torch.Tensor)
                             else yv, dtype=torch.float64).to(_dev()).reshape(-1)
        if yt.numel() != n:
            raise ValueError(f"X has {n} rows, y has {yt.numel()}")
        if not (torch.isfinite(Xc).all() and torch.isfinite(yt).all()):
            raise ValueError("Input contains NaN or infinity (as scikit-learn rejects it)")
        # Z = [x_1..x_p, y, r]: the residual column r drives the refinement passes
        Z = torch.cat([Xc, yt.view(1, -1), torch.zeros_like(yt).view(1, -1)], dim=0).contiguous()
        nseg = (n + SEG_ROWS - 1) // SEG_ROWS
        gram, shift = xs_gram(Z, n, SEG_ROWS, SEG_ROWS, list(range(p)), p, nseg=nseg,
                              row_limit=n)
        g, s = pool_moments(gram, shift, p)
        beta, nobs, rank = ols_solve(g, s, p, self.tol)
        # semi-normal equations + iterative refinement (accuracy ~ cond(X) eps instead of
        # cond(X)^2 eps, as scikit-learn's SVD-based lstsq): beta += C^-1 Xc' r
        L, P = _lib.lib(), _lib.ptr
        h = _lib.Context.get(Z.device.index).bind_stream()
        mean = s[0].contiguous()
        for _ in range(self.refine):
            _lib.check(L.afm_ols_residual_f64(h, P(Z), n, p, p, P(mean), P(beta[0]), P(Z[p + 1])),
                       "ols_residual")
            gr, sr = xs_gram(Z, n, SEG_ROWS, SEG_ROWS, list(range(p)), p + 1, nseg=nseg,
                             row_limit=n)
            g2, s2 = pool_moments(gr, sr, p)
            delta, _, _ = ols_solve(g2, s2, p, self.tol)
            _lib.check(L.afm_vec_add_f64(h, p, P(delta[0, 1:].contiguous()),
                                         P(beta[0, 1:])), "vec_add")
        _lib.check(L.afm_ols_intercept_f64(h, p, P(mean), P(beta[0])), "ols_intercept")
        b = beta[0].cpu().numpy()
        self.rank_ = int(rank[0].item())
        self.n_features_in_ = p
        if names is not None:
            self.feature_names_in_ = names
        if y2d:
            self.coef_ = b[1:].reshape(1, p)
            self.intercept_ = b[:1].copy()
        else:
            self.coef_ = b[1:].copy()
            self.intercept_ = float(b[0])
        self._beta = beta[0].contiguous()
        self._y2d = y2d
        return self

    def predict(self, X):
        import torch
        Xc, n, p, _ = self._as_columns(X)
        if p != self.n_features_in_:
            raise ValueError(f"X has {p} features, model was fit with {self.n_features_in_}")
        lda = (n + 63) // 64 * 64
        base = torch.zeros((p, lda), dtype=torch.float64, device=Xc.device)
        base[:, :n] = Xc
        bits = torch.zeros((1, lda), dtype=torch.int64, device=Xc.device)
        bits[0, :n] = 1
        out = predict_grid(base.view(p, 1, lda), lda, list(range(p)), self._beta, bits, 0, 1)
        pred = out[0, :n].cpu().numpy()
        return pred.reshape(-1, 1) if self._y2d else pred


class ConvergenceWarning(UserWarning):
    """Coordinate descent stopped at max_iter with the duality gap above tolerance (the
    condition under which scikit-learn warns)."""


class Lasso:
    """Drop-in for ``sklearn.linear_model.Lasso`` as the reference uses it
    (``Lasso(alpha=2e-4, max_iter=10000).fit(X_trainvalid, y_trainvalid)``, KKT:605-607).

    Minimises ``(1 / (2 n)) ||y - X w - b||^2 + alpha ||w||_1``.  The design's centered moments
    come from the same device Gram + Chan pooling as ``LinearRegression``; the fit is cyclic
    coordinate descent on them (``afm_lasso_cd_f64``: sklearn's Gram coordinate descent with
    its stopping rule and duality gap).  Results: ``coef_`` (p,), ``intercept_`` (float, or a
    1-element array for a one-column DataFrame / 2-D y, as sklearn), ``n_iter_``,
    ``dual_gap_`` (gap / n), ``n_features_in_``, ``feature_names_in_``."""

    def __init__(self, alpha: float = 1.0, *, fit_intercept: bool = True, precompute=False,
                 copy_X: bool = True, max_iter: int = 1000, tol: float = 1e-4,
                 warm_start: bool = False, positive: bool = False, random_state=None,
                 selection: str = "cyclic"):
        if not fit_intercept:
            raise NotImplementedError("only fit_intercept=True (the reference's usage)")
        if selection != "cyclic":
            raise NotImplementedError("only selection='cyclic' (the reference's usage)")
        if warm_start:
            raise NotImplementedError("warm_start is not supported")
        if alpha < 0 or tol < 0 or max_iter < 1:
            raise ValueError("alpha and tol must be >= 0 and max_iter >= 1")
        self.alpha = float(alpha)
        self.fit_intercept = True
        self.precompute = precompute
        self.copy_X = copy_X
        self.max_iter = int(max_iter)
        self.tol = float(tol)
        self.warm_start = False
        self.positive = bool(positive)
        self.random_state = random_state
        self.selection = selection

    def fit(self, X, y):
        import warnings

        import torch
        Xc, n, p, names = LinearRegression._as_columns(X)
        yv = y.to_numpy(dtype=np.float64) if hasattr(y, "to_numpy") else y
        y2d = getattr(yv, "ndim", 1) == 2
        yt = torch.as_tensor(np.asarray(yv, dtype=np.float64) if not isinstance(yv, torch.Tensor)
                             else yv, dtype=torch.float64).to(_dev()).reshape(-1)
        if yt.numel() != n:
            raise ValueError(f"X has {n} rows, y has {yt.numel()}")
        if not (torch.isfinite(Xc).all() and torch.isfinite(yt).all()):
            raise ValueError("Input contains NaN or infinity (as scikit-learn rejects it)")
        if self.alpha == 0:
            warnings.warn("With alpha=0 this is ordinary least squares by coordinate descent; "
                          "LinearRegression is the better tool.", UserWarning)
        Z = torch.cat([Xc, yt.view(1, -1)], dim=0).contiguous()
        nseg = (n + SEG_ROWS - 1) // SEG_ROWS
        gram, shift = xs_gram(Z, n, SEG_ROWS, SEG_ROWS, list(range(p)), p, nseg=nseg,
                              row_limit=n)
        g, s = pool_moments(gram, shift, p)
        w = torch.empty(p, dtype=torch.float64, device=Z.device)
        info = torch.empty(3, dtype=torch.float64, device=Z.device)
        h = _lib.Context.get(Z.device.index).bind_stream()
        _lib.check(_lib.lib().afm_lasso_cd_f64(h, _lib.ptr(g), p, self.alpha * n, 0.0,
                                               self.max_iter, self.tol, int(self.positive),
                                               _lib.ptr(w), _lib.ptr(info)), "afm_lasso_cd_f64")
        G = g[0].cpu().numpy()
        mean = s[0].cpu().numpy()[1:] + G[0, 1:] / G[0, 0]
        gap, tol_y, n_iter = info.cpu().numpy()
        self.coef_ = w.cpu().numpy()
        x_off, y_off = mean[:p], mean[p]
        icpt = y_off - np.dot(x_off, self.coef_)                 # sklearn _set_intercept
        self.intercept_ = np.array([icpt]) if y2d else float(icpt)
        self.n_iter_ = int(n_iter)
        self.dual_gap_ = float(gap) / n
        self.n_features_in_ = p
        if names is not None:
            self.feature_names_in_ = names
        if self.n_iter_ >= self.max_iter and not gap < tol_y:
            warnings.warn(f"Objective did not converge. Duality gap: {gap:.3e}, tolerance: "
                          f"{tol_y:.3e}", ConvergenceWarning)
        b = np.concatenate([[icpt], self.coef_])
        self._beta = torch.from_numpy(b).to(Z.device)
        return self

    def predict(self, X):
        import torch
        Xc, n, p, _ = LinearRegression._as_columns(X)
        if p != self.n_features_in_:
            raise ValueError(f"X has {p} features, model was fit with {self.n_features_in_}")
        lda = (n + 63) // 64 * 64
        base = torch.zeros((p, lda), dtype=torch.float64, device=Xc.device)
        base[:, :n] = Xc
        bits = torch.zeros((1, lda), dtype=torch.int64, device=Xc.device)
        bits[0, :n] = 1
        out = predict_grid(base.view(p, 1, lda), lda, list(range(p)), self._beta, bits, 0, 1)
        return out[0, :n].cpu().numpy()
