"""ORACLE -- test infrastructure only (see oracle/__init__.py): the CPU BASELINE leg.

The benchmarked chain restated in the reference's own CALL PATTERN -- pandas objects and the
library calls the notebook makes, one security / one date at a time -- so that bench.py can time
"the reference's CPU path" on the GPU box, where the reference itself cannot travel:

* compute_factors   per-security ``groupby`` loop of pandas rolling / ewm / diff / pct_change /
                    cumsum / rolling-corr column assignments, ``concat`` + ``dropna``
                    (No-talib.py:1-93)
* split + z-score   inclusive ``.loc`` date slices, ``columns.difference``, ``groupby`` mean /
                    std, ``(x - mu) / sigma``, inf -> NaN, ``dropna`` (KKT:424-458)
* Lasso             scikit-learn ``Lasso(alpha=2e-4, max_iter=10000)`` fit / predict (KKT:605-612)
* analyzer          per-id forward returns, merge, per-date demean, ``groupby`` Pearson IC,
                    pct ranks -> decile layers, top-10 factor-weighted returns (KKT:308-375)
* portfolio         per rebalance date: the ``in_trading_universe == 'Y'`` filter of all_df,
                    set intersection, ``nlargest`` / ``nsmallest``, history ``unstack``, ``cov``,
                    scipy SLSQP (min volatility, sum 1, 0 <= w <= 0.1), index-aligned turnover and
                    the value recursion (KKT:842-892), with the north-star rolling window

Written from the semantics in SURVEY.md §8(a); tests/test_pandas_chain.py checks its factor panel
against the C restatement (bit-exact) and its books against oracle/chain.py.
"""
from __future__ import annotations

import time

import numpy as np

SMA_W = range(6, 51, 4)
BB_W = range(14, 61, 6)


def _factors_one(df):
    """The 98 columns for one security's rows (date order)."""
    import pandas as pd
    c, v = df["close_price"], df["volume"]
    cols = {}
    for i in SMA_W:
        cols[f"SMA_{i}"] = c.rolling(i).mean()
    for i in SMA_W:
        cols[f"EMA_{i}"] = c.ewm(span=i, adjust=False).mean()
    vc = v * c
    for i in SMA_W:
        cols[f"VWMA_{i}"] = vc.rolling(i).mean() / v.rolling(i).mean()
    for i in BB_W:
        ma, sd = c.rolling(i).mean(), c.rolling(i).std()
        cols[f"BBANDS_upper_{i}"] = ma + 2 * sd
        cols[f"BBANDS_lower_{i}"] = ma - 2 * sd
    mom = {i: c.diff(i) for i in BB_W}
    for i in BB_W:
        cols[f"MOM_{i}"] = mom[i]
    for i in BB_W:
        cols[f"ACCEL_{i}"] = mom[i].diff()
    for i in BB_W:
        cols[f"ROCR_{i}"] = c.pct_change(i)
    e12 = c.ewm(span=12, adjust=False).mean()
    for i in (18, 24, 30):
        cols[f"MACD_12_{i}"] = e12 - c.ewm(span=i, adjust=False).mean()
    d = c.diff()
    up, down = d.clip(lower=0), -d.clip(upper=0)
    for i in (8, 14, 20):
        rs = up.ewm(com=i - 1, adjust=False).mean() / down.ewm(com=i - 1, adjust=False).mean()
        cols[f"RSI_{i}"] = 100 - 100 / (1 + rs)
    ret = c.pct_change()
    cols["PVT"] = (v * ret).cumsum()
    cols["OBV"] = (v * ((~d.le(0)) * 2 - 1)).cumsum()
    cols["PSY"] = (c > c.shift(1)).rolling(14).sum() / 14 * 100
    for i in (3, 5, 15):
        cols[f"sd_{i}"] = ret.rolling(i).std()
    cols["sd5_15"] = cols["sd_5"] / cols["sd_15"]
    for i in (3, 5, 15):
        cols[f"volsd_{i}"] = v.rolling(i).std()
    cols["volsd5_15"] = cols["volsd_5"] / cols["volsd_15"]
    vch = v.pct_change()
    cols["vol_change"] = vch
    for i in (5, 15):
        cols[f"corr_{i}"] = ret.rolling(i).corr(vch)
    cols["target"] = df["excess_ret1d"].shift(-1)
    cols["tmr_ret1d"] = df["ret1d"].shift(-1)
    return pd.concat([df, pd.DataFrame(cols, index=df.index)], axis=1)


def compute_factors(data):
    import pandas as pd
    data = data.sort_values(by=["security_id", "data_date"])
    parts = [_factors_one(df.sort_values("data_date"))
             for _, df in data.groupby("security_id")]
    return pd.concat(parts, ignore_index=True).dropna()


def _analyzer(pred, price, k_layers=10, top=10):
    """IC series, decile layer returns and top-10 backtest of ``pred`` [(date, id) -> value]."""
    import pandas as pd
    df = pred.to_frame("f")
    px = price.reset_index()
    for k in (1, 2, 5):
        r = px.groupby("id")["close_price"].apply(lambda s: s.pct_change(k).shift(-k))
        r = r.droplevel(0) if isinstance(r.index, pd.MultiIndex) else r
        ret = pd.Series(r.values, index=pd.MultiIndex.from_arrays([px["date"], px["id"]],
                                                                 names=["date", "id"]))
        ret = ret[ret <= 1]
        df = df.join(ret.rename(f"return_{k}"), how="inner").dropna()
        df[f"return_{k}"] = df[f"return_{k}"] - df.groupby(level="date")[f"return_{k}"].transform("mean")
    ic = df.groupby(level="date").apply(lambda x: x.corr()["f"].drop("f"))
    rank = df.groupby(level="date")["f"].rank(pct=True, method="first")
    layer = np.minimum((rank * k_layers).astype(int) + 1, k_layers)
    lay = df.assign(layer=layer).groupby([pd.Grouper(level="date"), "layer"]).mean().unstack()
    rk = df.groupby(level="date")["f"].rank(ascending=False, method="first")
    topd = df[rk <= top]
    w = topd["f"] / topd.groupby(level="date")["f"].transform("sum")
    port = topd.drop(columns="f").mul(w, axis=0).groupby(level="date").sum().cumsum()
    return ic, lay.cumsum(), port


def run_chain(p, train_end, valid_end, *, window=252, top_n=10, rate=1e-4, timings=None,
              max_dates=None):
    """The chain on synthetic panel ``p`` in the reference's call pattern; returns the value path.
    ``max_dates``: stop the per-date PortfolioManager loop after that many rebalance dates (a
    bounded timing sample; ``timings['dates']`` / ``['dates_total']`` say how many ran)."""
    import pandas as pd
    import scipy.optimize as sco
    from sklearn.linear_model import Lasso
    from afm.synthetic import to_frame
    tm = timings if timings is not None else {}
    t0 = time.perf_counter()
    fac = compute_factors(to_frame(p))
    all_df = fac.set_index(["data_date", "security_id"]).sort_index()
    tm["factors"] = time.perf_counter() - t0
    t1 = time.perf_counter()
    te, ve = pd.to_datetime(train_end), pd.to_datetime(valid_end)
    drop = ["close_price", "excess_ret1d", "group_id", "in_trading_universe", "ret1d", "volume",
            "target"]
    sets = {"train": all_df.loc[:te], "valid": all_df.loc[te:ve], "test": all_df.loc[ve:]}
    xs = {k: v[v.columns.difference(drop)] for k, v in sets.items()}
    mu = xs["train"].groupby(level="security_id").mean()
    sigma = xs["train"].groupby(level="security_id").std()
    for k, x in xs.items():
        z = (x - mu.reindex(x.index.get_level_values(1)).values) / \
            sigma.reindex(x.index.get_level_values(1)).values
        xs[k] = z.replace([np.inf, -np.inf], np.nan).dropna()
    ys = {k: sets[k].loc[xs[k].index, ["target"]] for k in xs}
    tm["zscore"] = time.perf_counter() - t1
    t2 = time.perf_counter()
    las = Lasso(alpha=2e-4, max_iter=10000).fit(pd.concat([xs["train"], xs["valid"]]),
                                                 pd.concat([ys["train"], ys["valid"]]))
    pred = pd.Series(las.predict(xs["test"]), index=xs["test"].index)
    pred.index.names = ["date", "id"]
    tm["lasso"] = time.perf_counter() - t2
    t3 = time.perf_counter()
    price = sets["test"][["close_price"]].copy()
    price.index.names = ["date", "id"]
    _analyzer(pred, price)
    tm["analyzer"] = time.perf_counter() - t3
    t4 = time.perf_counter()
    hist = pd.concat([ys["train"], ys["valid"], ys["test"]])["target"]
    hist = hist[~hist.index.duplicated()]
    calendar = all_df.index.get_level_values(0).unique()
    value, cur = [100000000.0], None

    def weights(R):
        cov = R.cov()
        n = len(cov)
        res = sco.minimize(lambda w: np.sqrt(w @ cov.values @ w), n * [1.0 / n],
                           method="SLSQP", bounds=[(0, 0.1)] * n,
                           constraints=({"type": "eq", "fun": lambda x: np.sum(x) - 1},))
        return res["x"]

    t_filter = 0.0
    groups = pred.groupby(level="date")
    tm["dates_total"] = groups.ngroups
    tm["dates"] = 0
    for date, preds in groups:
        if max_dates is not None and tm["dates"] >= max_dates:
            break
        tm["dates"] += 1
        preds = preds.droplevel(0)
        tf = time.perf_counter()
        trad = all_df[all_df["in_trading_universe"] == "Y"].loc[date].index     # KKT:847, O(panel)
        t_filter += time.perf_counter() - tf
        ids = list(set(trad) & set(preds.index))
        k = len(ids) // 2 if len(ids) < 2 * top_n else top_n
        longs = preds.loc[ids].nlargest(k).index.tolist()
        shorts = preds.loc[ids].nsmallest(k).index.tolist()
        j = calendar.get_loc(date)
        lo = calendar[max(0, j - window)]
        h = hist.loc[lo:date]
        h = h[h.index.get_level_values(0) < date]
        wl = weights(h[h.index.get_level_values(1).isin(longs)].unstack())
        ws = weights(h[h.index.get_level_values(1).isin(shorts)].unstack())
        day = all_df.loc[date]
        r = ((day.loc[longs, "tmr_ret1d"] * wl).sum() - (day.loc[shorts, "tmr_ret1d"] * ws).sum()) / 2
        size = value[-1] / 2
        new = pd.Series(np.nan, index=preds.index)
        new[longs] = size / sum(wl * day.loc[longs, "close_price"])
        new[shorts] = -size / sum(ws * day.loc[shorts, "close_price"])
        turn = 0.0 if cur is None else (cur.fillna(0) - new.fillna(0)).abs().sum() / 2
        r -= turn * rate / value[-1]
        value.append(value[-1] * (1 + r))
        cur = new
    tm["portfolio"] = time.perf_counter() - t4
    tm["filter_847"] = t_filter                      # inside "portfolio": the per-date all_df filter
    return np.array(value)
