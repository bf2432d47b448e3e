"""Signal evaluation -- drop-in for ``AlphaSignalAnalyzer`` ("KKT Yuliang Jiang.py":280-419),
SURVEY.md §8(a) rows A1-A4.

``run()`` evaluates forward returns, the per-date demean cascade, IC/IR, decile layers and the
top-10 backtest on the GPU (csrc/analyzer.hip) and rebuilds the reference's attributes
(``factor_df``, ``ic_df``, ``ir_df``, ``layered_ret_dfs``, ``ls_ret_dfs``, ``port_ret_df``,
``port_df``) with the same columns, row order and values (bit-exact with pandas 2.3.3).
Plotting (``_gen_report``, KKT:377-419) is out of scope and does nothing.  ``ic_df`` carries a
fresh RangeIndex (the reference's keeps the gaps of its dropped 'id' rows).
"""
from __future__ import annotations

import numpy as np

from . import _lib
from .grid import pack_bits

RETURN_TYPES = ["return_1", "return_2", "return_5"]


def _dev():
    import torch
    return torch.device("cuda", torch.cuda.current_device())


def evaluate_grid(sig, close, price_bits, *, A: int, dates_idx=None, year=None):
    """Device-level A1-A4 on grids: ``sig`` [T][lda] (NaN = no row), ``close`` [T][lda] with
    ``price_bits`` presence.  Returns a dict of device tensors."""
    import torch
    dev = sig.device
    T, lda = sig.shape
    plane = T * lda
    ctx = _lib.Context.get(dev.index)
    P = _lib.ptr
    L = _lib.lib()
    h = ctx.bind_stream()
    fr = torch.empty((3, T, lda), dtype=torch.float64, device=dev)
    _lib.check(L.afm_fwd_returns_f64(h, T, lda, P(close), P(price_bits), P(fr)), "fwd_returns")
    scratch = torch.empty((T, lda), dtype=torch.float64, device=dev)
    rows = torch.empty((4, T, lda), dtype=torch.float64, device=dev)
    rows_idx = torch.empty((T, lda), dtype=torch.int32, device=dev)
    nrows = torch.empty(T, dtype=torch.int32, device=dev)
    _lib.check(L.afm_xs_prepare_f64(h, T, A, lda, P(sig), P(fr), P(scratch), P(rows), P(rows_idx),
                                    P(nrows)), "xs_prepare")
    skey = torch.empty((T, lda), dtype=torch.int64, device=dev)
    sidx = torch.empty((T, lda), dtype=torch.int32, device=dev)
    ra = torch.empty((T, lda), dtype=torch.int32, device=dev)
    rd = torch.empty((T, lda), dtype=torch.int32, device=dev)
    _lib.check(L.afm_xs_rank_f64(h, T, lda, P(rows), P(nrows), P(skey), P(sidx), P(ra), P(rd)),
               "xs_rank")
    nr = nrows.cpu().numpy()
    if dates_idx is None:
        dates_idx = np.flatnonzero(nr > 0).astype(np.int32)
    nd = len(dates_idx)
    mcols = int(min(10, nr[dates_idx].max())) if nd else 0
    d_t = torch.from_numpy(np.ascontiguousarray(dates_idx, dtype=np.int32)).to(dev)
    ic = torch.empty((nd, 3), dtype=torch.float64, device=dev)
    lm = torch.empty((nd, 3, 10), dtype=torch.float64, device=dev)
    lc = torch.empty((nd, 10), dtype=torch.int32, device=dev)
    port = torch.empty((nd, 3), dtype=torch.float64, device=dev)
    _lib.check(L.afm_xs_stats_f64(h, T, lda, P(d_t), nd, P(rows), P(nrows), P(ra), P(rd), mcols,
                                  P(ic), P(lm), P(lc), P(port)), "xs_stats")
    out = {"fr": fr, "rows": rows, "rows_idx": rows_idx, "nrows": nrows, "rank_asc": ra,
           "rank_desc": rd, "dates_idx": dates_idx, "ic": ic, "layer_mean": lm,
           "layer_cnt": lc, "port": port, "mcols": mcols}
    if year is not None and nd:
        yr = np.asarray(year, dtype=np.int32)[dates_idx]
        y0, ny = int(yr.min()), int(yr.max() - yr.min() + 1)
        y_t = torch.from_numpy(np.ascontiguousarray(yr)).to(dev)
        cum_layer = torch.empty_like(lm)
        ls = torch.empty((nd, 3, 5), dtype=torch.float64, device=dev)
        cum_port = torch.empty_like(port)
        ir = torch.empty((ny, 3), dtype=torch.float64, device=dev)
        scr = torch.empty((3 * ny, nd), dtype=torch.float64, device=dev)
        _lib.check(L.afm_xs_series_f64(h, nd, P(lm), P(port), P(ic), P(y_t), ny, y0,
                                       P(cum_layer), P(ls), P(cum_port), P(ir), P(scr)),
                   "xs_series")
        out.update(cum_layer=cum_layer, ls=ls, cum_port=cum_port, ir=ir, year0=y0, years=yr)
    return out


class AlphaSignalAnalyzer:
    """Drop-in for ``AlphaSignalAnalyzer`` (KKT:280-419)."""

    def __init__(self, alpha_signal_df, factor_name: str, price_data):
        self.factor_df = alpha_signal_df
        self.factor_df.index.names = ["date", "id"]                  # KKT:283
        self.factor_name = factor_name
        self.corr_method = "pearson"
        self.k_layers = 10
        self.portfolio_stock_num = 10
        self.return_type = list(RETURN_TYPES)
        self.price_data = price_data
        self.price_data.index.names = ["date", "id"]                 # KKT:292
        self.price_data = self.price_data.reset_index()
        self.layered_ret_dfs = dict()
        self.ls_ret_dfs = dict()
        self._res = None

    def run(self):                                                   # KKT:298-306
        print("-" * 50)
        print("Running analysis...")
        self._add_returns()
        self._calc_sdav_ic()
        for layered_ret_type in self.return_type:
            self._calc_layered_ret(layered_ret_type)
        self._backtest_top_stocks()
        self._gen_report()

    # -- the GPU evaluation, run once ---------------------------------------------------------
    def _evaluate(self):
        import torch
        fd = self.factor_df.reset_index()
        sd = fd["date"].to_numpy().astype("datetime64[ns]")
        si = fd["id"].to_numpy().astype(np.int64)
        sv = fd[self.factor_name].to_numpy(np.float64)
        pd_ = self.price_data["date"].to_numpy().astype("datetime64[ns]")
        pi_ = self.price_data["id"].to_numpy().astype(np.int64)
        pc = self.price_data["close_price"].to_numpy(np.float64)
        dates = np.unique(np.concatenate([sd, pd_]))
        ids = np.unique(np.concatenate([si, pi_]))
        T, A = len(dates), len(ids)
        lda = (A + 63) // 64 * 64
        dev = _dev()

        def scatter(d, i, v):
            g = torch.full((T, lda), float("nan"), dtype=torch.float64, device=dev)
            ti = torch.from_numpy(np.searchsorted(dates, d)).to(dev)
            ai = torch.from_numpy(np.searchsorted(ids, i)).to(dev)
            g[ti, ai] = torch.from_numpy(np.ascontiguousarray(v)).to(dev)
            return g, ti, ai

        sig, _, _ = scatter(sd, si, sv)
        close, ti, ai = scatter(pd_, pi_, pc)
        pm = torch.zeros((T, lda), dtype=torch.bool, device=dev)
        pm[ti, ai] = True
        year = dates.astype("datetime64[Y]").astype(np.int64) + 1970
        res = evaluate_grid(sig, close, pack_bits(pm), A=A, year=year)
        res["dates"], res["ids"] = dates, ids
        self._res = res

    def _add_returns(self):                                          # KKT:308-320
        import pandas as pd
        print("Adding returns...")
        self._evaluate()
        r = self._res
        nr = r["nrows"].cpu().numpy()
        di = r["dates_idx"]
        rows = r["rows"].cpu().numpy()
        ridx = r["rows_idx"].cpu().numpy()
        dd, ii, vals = [], [], []
        for t in di:
            n = nr[t]
            dd.append(np.full(n, t))
            ii.append(ridx[t, :n])
            vals.append(rows[:, t, :n].T)
        dd = np.concatenate(dd) if dd else np.zeros(0, np.int64)
        ii = np.concatenate(ii) if ii else np.zeros(0, np.int64)
        vals = np.concatenate(vals) if vals else np.zeros((0, 4))
        idx = pd.MultiIndex.from_arrays([pd.DatetimeIndex(r["dates"][dd]), r["ids"][ii]],
                                        names=["date", "id"])
        self.factor_df = pd.DataFrame(vals, index=idx,
                                      columns=[self.factor_name] + self.return_type)

    def _calc_sdav_ic(self):                                         # KKT:342-354
        import pandas as pd
        print("Calculating IC & IR...")
        r = self._res
        ic = r["ic"].cpu().numpy()
        dts = pd.DatetimeIndex(r["dates"][r["dates_idx"]])
        d, ty, v = [], [], []
        for i in range(len(dts)):
            for k, rt in enumerate(self.return_type):
                if ic[i, k] == ic[i, k]:
                    d.append(dts[i]); ty.append(rt); v.append(ic[i, k])
        self.ic_df = pd.DataFrame({"date": d, "Type": ty, "IC": np.asarray(v, dtype=np.float64)})
        self.ic_df["year"] = self.ic_df["date"].apply(lambda x: x.year)
        ir = r["ir"].cpu().numpy() if "ir" in r else np.zeros((0, 3))
        present = {(y, t) for y, t in zip(self.ic_df["year"], self.ic_df["Type"])}
        rows = [(r["year0"] + y, rt, ir[y, k]) for y in range(ir.shape[0])
                for k, rt in enumerate(self.return_type) if (r["year0"] + y, rt) in present]
        self.ir_df = pd.DataFrame(rows, columns=["year", "Type", "IR"])

    def _calc_layered_ret(self, layered_ret_type):                   # KKT:324-340
        import pandas as pd
        print(f"Calculating layered return of {layered_ret_type}...")
        r = self._res
        k = self.return_type.index(layered_ret_type)
        cum = r["cum_layer"][:, k, :].cpu().numpy()
        cnt = r["layer_cnt"].cpu().numpy()
        ls = r["ls"][:, k, :].cpu().numpy()
        dts = pd.DatetimeIndex(r["dates"][r["dates_idx"]])
        layers = np.flatnonzero((cnt > 0).any(axis=0)) + 1
        d, l, v = [], [], []
        for i in range(len(dts)):
            for ly in layers:
                x = cum[i, ly - 1]
                if x == x:
                    d.append(dts[i]); l.append(ly); v.append(x)
        self.layered_ret_dfs[layered_ret_type] = pd.DataFrame(
            {"date": d, "layer": np.asarray(l, dtype=np.int64), layered_ret_type: np.asarray(v)})
        d, l, v = [], [], []
        half = self.k_layers // 2
        for i in range(len(dts)):
            for lyr in range(1, half + 1):
                x = ls[i, lyr - 1]
                if x == x:
                    d.append(dts[i]); l.append(half - lyr + 1); v.append(x)
        self.ls_ret_dfs[layered_ret_type] = pd.DataFrame(
            {"date": d, "layer": np.asarray(l, dtype=np.int64), layered_ret_type: np.asarray(v)})

    def _backtest_top_stocks(self):                                  # KKT:356-375
        import pandas as pd
        print("Backtesting top stocks...")
        r = self._res
        port = r["port"].cpu().numpy()
        cum = r["cum_port"].cpu().numpy()
        dts = pd.DatetimeIndex(r["dates"][r["dates_idx"]])
        names = self.return_type + [f"cum_{x}" for x in self.return_type]
        full = np.concatenate([port, cum], axis=1)
        self.port_ret_df = pd.DataFrame({
            "date": np.repeat(dts.values, len(names)),
            "Type": np.tile(np.asarray(names, dtype=object), len(dts)),
            "Returns": full.reshape(-1)})
        # the selected rows, sorted by (date, rank), rank as str (KKT:358-362)
        rd = r["rank_desc"].cpu().numpy()
        nr = r["nrows"].cpu().numpy()
        ridx = r["rows_idx"].cpu().numpy()
        rows = r["rows"].cpu().numpy()
        recs = []
        for t in r["dates_idx"]:
            n = nr[t]
            sel = np.flatnonzero(rd[t, :n] <= self.portfolio_stock_num)
            sel = sel[np.argsort(rd[t, sel], kind="stable")]
            for e in sel:
                recs.append((r["dates"][t], r["ids"][ridx[t, e]], *rows[:, t, e], float(rd[t, e])))
        self.port_df = pd.DataFrame(recs, columns=["date", "id", self.factor_name] +
                                    self.return_type + ["rank"])
        self.port_df["date"] = pd.to_datetime(self.port_df["date"])
        self.port_df["rank"] = self.port_df["rank"].astype(str)

    def _gen_report(self):                                           # KKT:377-419 (plots)
        """Plotting is out of scope; the frames above are the results."""
        print("Generating report...")
