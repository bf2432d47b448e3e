"""Golden vectors of the reference chain at BASELINE config A (500 assets x 10 years) from the
CPU oracle (oracle/chain.py): the slow pieces (PortfolioManager with the exact QP, the analyzer,
the per-date FM regressions) are stored so the GPU test only re-runs the fast ones live.

    python tests/golden/make_chain_golden.py      # writes tests/golden/chain_A.npz (~40 s)
"""
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]

# config A (BASELINE.json configs[0]): the reference CPU run's panel; split dates inside the
# synthetic 2000-2009 calendar, train_end a trading day (its rows enter the fit twice, as the
# reference's 2015-12-31), valid_end a trading day (in valid and test)
CONFIG_A = dict(assets=500, days=2520, seed=2023, tradable_p=0.9, train_end="2006-12-29",
                valid_end="2007-12-31", window=252, top_n=10)


def main():
    from afm.pipeline import FM30
    from afm.synthetic import make_panel
    from oracle import chain
    c = CONFIG_A
    p = make_panel(c["assets"], c["days"], seed=c["seed"], tradable_p=c["tradable_p"])
    r = chain.run_chain(p, c["train_end"], c["valid_end"], fm_features=FM30, top_n=c["top_n"],
                        window=c["window"])
    pr, an = r["portfolio"], r["analyzer"]
    books = np.full((len(pr["dates"]), 2, c["top_n"]), -1, np.int32)
    weights = np.zeros((len(pr["dates"]), 2, c["top_n"]))
    for i in range(len(pr["dates"])):
        for s in range(2):
            b, w = pr["books"][2 * i + s], pr["weights"][2 * i + s]
            books[i, s, :len(b)] = b
            weights[i, s, :len(w)] = w
    np.savez_compressed(
        os.path.join(HERE, "chain_A.npz"),
        coef=r["coef"], intercept=r["intercept"], n_fit=r["n_fit"], n_iter=r["n_iter"],
        reb_dates=pr["dates"], books=books, weights=weights, value=pr["value"],
        turnover=pr["turnover"], long_ret=pr["long_ret"], short_ret=pr["short_ret"],
        ic_date=an["ic_date"], ic_type=an["ic_type"].astype("U8"), ic=an["ic"],
        ir_year=an["ir_year"], ir=an["ir"], pt_ret=an["pt_ret"],
        lay1=an["lay_return_1"], ls1=an["ls_return_1"],
        fm_dates=r["fm_dates"], fm_beta=r["fm_beta"], fm_n=r["fm_n"])
    print("chain_A.npz:", len(pr["dates"]), "rebalance dates, final value", pr["value"][-1])


if __name__ == "__main__":
    main()
