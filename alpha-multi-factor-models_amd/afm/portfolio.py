"""Rebalance, weights and PnL -- drop-in for ``PortfolioManager`` ("KKT Yuliang Jiang.py":795-970),
SURVEY.md §8(a) rows K1-K4.

``calculate_portfolio`` runs every rebalance date in one GPU launch (csrc/portfolio.hip:
selection, pairwise-complete history covariance, exact box-QP weights, PnL components) followed
by the sequential value/turnover scan, and fills the reference's attributes
(``portfolio_value['Portfolio']``, ``turnovers``, ``long_returns``, ``short_returns``,
``current_positions``, ``positions``).  ``determine_weights`` solves one book.

Differences from the reference, by design:
* weights are the EXACT optimum of min w'Sw, sum w = 1, 0 <= w <= 0.1 (SLSQP stops ~1e-3 short
  when bounds bind); at the default top_n = 10 both are 0.1 exactly;
* equal predictions are ordered by ascending security id (the reference: Python set order).
Extensions: ``window`` (rolling history window in dates; None = the reference's whole history),
``books`` (the long/short ids per date -- the reference's ``positions`` stays all-NaN because its
chained assignment at KKT:890-891 never writes).
"""
from __future__ import annotations

import numpy as np

from . import _lib

V0 = 100000000
MAX_BOOK = 128


def _dev():
    import torch
    return torch.device("cuda", torch.cuda.current_device())


def rebalance(pred, trad_bits, hist, hist_bits, close, tmr, dates_idx, *, A: int, top_n: int = 10,
              window: int | None = None, h_range=None, lo: float = 0.0, hi: float = 0.1):
    """Device-level K1-K3 for the grid panel.  All arrays torch CUDA tensors ([T][lda] planes,
    [ceil(T/64)][lda] bit words); ``dates_idx`` int32 grid indices of the rebalance dates.
    Returns a dict of device tensors (k, books, weights, sums, upos, usize, status)."""
    import torch
    dev = pred.device
    T, lda = pred.shape
    nd = int(dates_idx.numel())
    out = {
        "k": torch.empty(nd, dtype=torch.int32, device=dev),
        "books": torch.full((nd, 2, MAX_BOOK), -1, dtype=torch.int32, device=dev),
        "weights": torch.zeros((nd, 2, MAX_BOOK), dtype=torch.float64, device=dev),
        "sums": torch.empty((nd, 4), dtype=torch.float64, device=dev),
        "upos": torch.empty((nd, 2, 2, MAX_BOOK), dtype=torch.int32, device=dev),
        "usize": torch.empty((nd, 2), dtype=torch.int64, device=dev),
        "status": torch.empty(nd, dtype=torch.int32, device=dev),
    }
    h0, h1 = h_range if h_range is not None else (0, T)
    ctx = _lib.Context.get(dev.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_rebalance_f64(
        ctx.bind_stream(), T, A, lda, P(dates_idx), nd, P(pred), P(trad_bits), P(hist),
        P(hist_bits), h0, h1, -1 if window is None else int(window), P(close), P(tmr), int(top_n),
        float(lo), float(hi), P(out["k"]), P(out["books"]), P(out["weights"]), P(out["sums"]),
        P(out["upos"]), P(out["usize"]), P(out["status"])), "afm_rebalance_f64")
    return out


def pnl_scan(reb: dict, v0: float = V0, rate: float = 1e-4):
    """Value/turnover recursion (KKT:864-892) -> dict of device tensors."""
    import torch
    nd = reb["k"].numel()
    dev = reb["k"].device
    res = {"value": torch.empty(nd + 1, dtype=torch.float64, device=dev),
           "turnover": torch.empty(nd, dtype=torch.float64, device=dev),
           "long_ret": torch.empty(nd, dtype=torch.float64, device=dev),
           "short_ret": torch.empty(nd, dtype=torch.float64, device=dev)}
    ctx = _lib.Context.get(dev.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_pnl_scan_f64(
        ctx.bind_stream(), nd, P(reb["k"]), P(reb["books"]), P(reb["sums"]), P(reb["upos"]),
        P(reb["usize"]), float(v0), float(rate), P(res["value"]), P(res["turnover"]),
        P(res["long_ret"]), P(res["short_ret"])), "afm_pnl_scan_f64")
    return res


def bootstrap_paths(nd: int, n_paths: int = 1024, steps: int | None = None, seed: int = 2023):
    """Rebalance-date slots drawn with replacement (BASELINE config E): int32 [n_paths][steps]."""
    steps = nd if steps is None else steps
    return np.random.default_rng(seed).integers(0, nd, size=(n_paths, steps)).astype(np.int32)


def bootstrap_pnl(reb: dict, pred, dates_idx, paths, v0: float = V0, rate: float = 1e-4):
    """Config E: the value/turnover recursion (KKT:864-892) over every bootstrap path of book
    slots (``paths`` [npaths][steps] into the dates of ``reb``), one workgroup per path ->
    dict of device tensors value [npaths][steps+1], turnover / long_ret / short_ret
    [npaths][steps]."""
    import torch
    dev = reb["k"].device
    paths = torch.as_tensor(np.asarray(paths, dtype=np.int32) if not torch.is_tensor(paths)
                            else paths, device=dev).to(torch.int32).contiguous()
    npaths, steps = int(paths.shape[0]), int(paths.shape[1])
    nd = int(reb["k"].numel())
    res = {"value": torch.empty((npaths, steps + 1), dtype=torch.float64, device=dev),
           "turnover": torch.empty((npaths, steps), dtype=torch.float64, device=dev),
           "long_ret": torch.empty((npaths, steps), dtype=torch.float64, device=dev),
           "short_ret": torch.empty((npaths, steps), dtype=torch.float64, device=dev)}
    ctx = _lib.Context.get(dev.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_bootstrap_pnl_f64(
        ctx.bind_stream(), int(pred.shape[1]), P(dates_idx), nd, P(pred), P(reb["k"]),
        P(reb["books"]), P(reb["sums"]), npaths, steps, P(paths), float(v0), float(rate),
        P(res["value"]), P(res["turnover"]), P(res["long_ret"]), P(res["short_ret"])),
        "afm_bootstrap_pnl_f64")
    return res


def min_variance_weights(returns, lo: float = 0.0, hi: float = 0.1):
    """determine_weights for one book: returns [rows][k] (NaN = missing) -> (w[k], cov[k][k])."""
    import torch
    R = torch.as_tensor(np.ascontiguousarray(np.asarray(returns, dtype=np.float64)),
                        device=_dev())
    if R.ndim != 2:
        raise ValueError("returns must be 2-D [dates x assets]")
    rows, k = R.shape
    if k > MAX_BOOK:
        raise ValueError(f"book of {k} > {MAX_BOOK} names")
    w = torch.empty(k, dtype=torch.float64, device=R.device)
    cov = torch.empty((k, k), dtype=torch.float64, device=R.device)
    st = torch.empty(1, dtype=torch.int32, device=R.device)
    ctx = _lib.Context.get(R.device.index)
    P = _lib.ptr
    _lib.check(_lib.lib().afm_min_variance_weights_f64(ctx.bind_stream(), P(R), rows, k, k,
                                                       float(lo), float(hi), P(w), P(cov),
                                                       P(st)), "afm_min_variance_weights_f64")
    return w.cpu().numpy(), cov.cpu().numpy()


class PortfolioManager:
    """Drop-in for ``PortfolioManager`` (KKT:795-970)."""

    def __init__(self, predictions, history, all_df, trading_cost_rate=0.0001, top_n=10,
                 window=None, lo=0.0, hi=0.1):
        import pandas as pd
        self.predictions = predictions
        self.predictions.index.names = ["date", "id"]              # KKT:798
        self.history = history
        self.history.index.names = ["date", "id"]                  # KKT:800
        self.all_df = all_df
        self.trading_cost_rate = trading_cost_rate
        self.top_n = top_n
        self.window = window
        self.lo, self.hi = lo, hi
        self.portfolio_value = {"Portfolio": [V0]}
        self.current_positions = pd.Series(index=self.predictions.columns, dtype=np.float64)
        self.turnovers = []
        self.positions = pd.DataFrame(index=predictions.index.levels[0], columns=["long", "short"])
        self.long_returns = []
        self.short_returns = []
        self.books = []

    def Portfolio_volatility(self, weights, mean_returns, cov_matrix):   # KKT:811-815
        return np.sqrt(np.dot(weights.T, np.dot(cov_matrix, weights)))

    def determine_weights(self, returns):                                # KKT:817-833
        w, _ = min_variance_weights(returns.to_numpy(np.float64) if hasattr(returns, "to_numpy")
                                    else returns, self.lo, self.hi)
        return w

    def _grid(self):
        import torch
        dev = _dev()
        pr, hs, ad = self.predictions, self.history, self.all_df

        def lv(f, k):
            return np.asarray(f.index.get_level_values(k).values)
        pd_, pi_ = lv(pr, 0).astype("datetime64[ns]"), lv(pr, 1).astype(np.int64)
        hd_, hi_ = lv(hs, 0).astype("datetime64[ns]"), lv(hs, 1).astype(np.int64)
        ad_, ai_ = lv(ad, 0).astype("datetime64[ns]"), lv(ad, 1).astype(np.int64)
        dates = np.unique(np.concatenate([pd_, hd_, ad_]))
        ids = np.unique(np.concatenate([pi_, hi_, ai_]))
        T, A = len(dates), len(ids)
        lda = (A + 63) // 64 * 64

        def scatter(d, i, vals, fill=float("nan")):
            g = torch.full((T, lda), fill, dtype=torch.float64, device=dev)
            ti = torch.from_numpy(np.searchsorted(dates, d)).to(dev)
            ai = torch.from_numpy(np.searchsorted(ids, i)).to(dev)
            g[ti, ai] = torch.from_numpy(np.ascontiguousarray(vals, dtype=np.float64)).to(dev)
            return g, ti, ai

        from .grid import pack_bits
        pred, _, _ = scatter(pd_, pi_, pr.iloc[:, 0].to_numpy(np.float64))
        hist, hti, hai = scatter(hd_, hi_, hs.iloc[:, 0].to_numpy(np.float64))
        hmask = torch.zeros((T, lda), dtype=torch.bool, device=dev)
        hmask[hti, hai] = True
        close, ti, ai = scatter(ad_, ai_, ad["close_price"].to_numpy(np.float64))
        tmr, _, _ = scatter(ad_, ai_, ad["tmr_ret1d"].to_numpy(np.float64))
        tmask = torch.zeros((T, lda), dtype=torch.bool, device=dev)
        tmask[ti, ai] = torch.from_numpy(ad["in_trading_universe"].to_numpy() == "Y").to(dev)
        rdates = np.searchsorted(dates, np.unique(pd_)).astype(np.int32)
        return dict(dates=dates, ids=ids, A=A, pred=pred, hist=hist, hbits=pack_bits(hmask),
                    close=close, tmr=tmr, tbits=pack_bits(tmask),
                    rdates=torch.from_numpy(rdates).to(dev), rdates_np=rdates)

    def calculate_portfolio(self):                                       # KKT:842-892
        import pandas as pd
        g = self._grid()
        reb = rebalance(g["pred"], g["tbits"], g["hist"], g["hbits"], g["close"], g["tmr"],
                        g["rdates"], A=g["A"], top_n=self.top_n, window=self.window, lo=self.lo,
                        hi=self.hi)
        res = pnl_scan(reb, V0, self.trading_cost_rate)
        st = reb["status"].cpu().numpy()
        if (st == 2).any():
            raise ValueError(f"top_n={self.top_n} exceeds the {MAX_BOOK}-name book limit")
        k = reb["k"].cpu().numpy()
        books = reb["books"].cpu().numpy()
        value = res["value"].cpu().numpy()
        to = res["turnover"].cpu().numpy()
        lr, sr = res["long_ret"].cpu().numpy(), res["short_ret"].cpu().numpy()
        ids = g["ids"]
        dts = g["dates"][g["rdates_np"]]
        self.weights = reb["weights"].cpu().numpy()
        for i in range(len(k)):
            L = ids[books[i, 0, :k[i]]].tolist()
            S = ids[books[i, 1, :k[i]]].tolist()
            self.books.append((pd.Timestamp(dts[i]), L, S))
            self.long_returns.append(lr[i])
            self.short_returns.append(sr[i])
            self.turnovers.append(0 if i == 0 else to[i])
            self.portfolio_value["Portfolio"].append(value[i + 1])
        if len(k):
            last = dts[-1]
            preds = self.predictions.xs(pd.Timestamp(last), level=0)
            pos = pd.Series(index=preds.index, dtype=np.float64)
            size = value[-2] / 2
            sm = reb["sums"][-1].cpu().numpy()
            _, L, S = self.books[-1]
            pos[L] = size / sm[2]
            pos[S] = -size / sm[3]
            self.current_positions = pos

    def bootstrap(self, n_paths: int = 1024, steps: int | None = None, seed: int = 2023,
                  paths=None):
        """Extension (BASELINE config E): re-run the rebalance loop over ``n_paths`` bootstrap
        resamples (with replacement) of the rebalance dates.  Books and weights per date are
        those of ``calculate_portfolio``; each path has its own turnover and value recursion.
        Returns (paths [n_paths][steps] indices into the sorted rebalance dates, dict of numpy
        arrays value [n_paths][steps+1], turnover, long_ret, short_ret [n_paths][steps])."""
        g = self._grid()
        reb = rebalance(g["pred"], g["tbits"], g["hist"], g["hbits"], g["close"], g["tmr"],
                        g["rdates"], A=g["A"], top_n=self.top_n, window=self.window, lo=self.lo,
                        hi=self.hi)
        nd = int(reb["k"].numel())
        if paths is None:
            paths = bootstrap_paths(nd, n_paths, steps, seed)
        res = bootstrap_pnl(reb, g["pred"], g["rdates"], paths, V0, self.trading_cost_rate)
        return np.asarray(paths), {k: v.cpu().numpy() for k, v in res.items()}

    def calculate_sharpe_ratio(self):                                    # KKT:894-897
        import pandas as pd
        returns = pd.Series(self.portfolio_value["Portfolio"]).pct_change().dropna()
        return returns.mean() / returns.std()

    def annualized_return(self):                                         # KKT:945-949
        total_return = self.portfolio_value["Portfolio"][-1] / self.portfolio_value["Portfolio"][0] - 1
        years = len(self.portfolio_value["Portfolio"]) / 252
        return (1 + total_return) ** (1 / years) - 1

    def max_drawdown(self):                                              # KKT:951-955
        import pandas as pd
        returns = np.array(self.portfolio_value["Portfolio"])
        running_max = pd.Series(returns).cummax().values
        drawdowns = (running_max - returns) / running_max
        return drawdowns.max()

    def position_overview(self):                                         # KKT:957-962
        long_positions = len(self.current_positions[self.current_positions == 1])
        short_positions = len(self.current_positions[self.current_positions == -1])
        print(f"Long Positions: {long_positions}")
        print(f"Short Positions: {short_positions}")

    def summary(self):                                                   # KKT:964-970
        print("Portfolio Summary")
        print("------------------")
        print(f"Sharpe Ratio: {self.calculate_sharpe_ratio():.3f}")
        print(f"Annualized Return: {self.annualized_return():.3f}")
        print(f"Maximum Drawdown: {self.max_drawdown():.3f}")
        self.position_overview()
