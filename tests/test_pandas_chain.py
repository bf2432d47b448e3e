"""oracle/pandas_chain.py (bench.py's cpu_baseline leg: the reference's CPU path in its own pandas
call pattern) against the C factor restatement and the vectorised oracle chain, on a small panel.
"""
import numpy as np
import pytest


@pytest.fixture(scope="module")
def panel():
    from afm.synthetic import make_panel
    return make_panel(24, 2520, seed=11, tradable_p=0.9)


def test_factor_loop_matches_c_restatement(panel):
    import oracle
    from afm.synthetic import to_frame
    from oracle import pandas_chain
    fac = pandas_chain.compute_factors(to_frame(panel))
    ref = oracle.compute_factors(to_frame(panel))
    assert len(fac) == len(ref)
    f = fac.sort_values(["data_date", "security_id"]).reset_index(drop=True)
    r = ref.sort_values(["data_date", "security_id"]).reset_index(drop=True)
    assert (f["security_id"].values == r["security_id"].values).all()
    for name in oracle.FACTOR_NAMES:
        a, b = f[name].to_numpy(np.float64), r[name].to_numpy(np.float64)
        np.testing.assert_allclose(a, b, rtol=1e-12, atol=1e-12 * np.abs(b).max(), err_msg=name)


def test_value_path_matches_oracle_chain(panel):
    from oracle import chain, pandas_chain
    import pandas as pd
    d = pd.to_datetime(panel.dates)
    te, ve = str(d[-140].date()), str(d[-80].date())          # 80 test dates keep this quick
    tm = {}
    for top_n, rtol in ((10, 1e-8), (3, 1e-4)):
        v = pandas_chain.run_chain(panel, te, ve, top_n=top_n, timings=tm)
        r = chain.run_chain(panel, te, ve, top_n=top_n, analyzer=False, fm=False)
        assert set(tm) == {"factors", "zscore", "lasso", "analyzer", "portfolio", "filter_847",
                           "dates", "dates_total"}
        assert tm["dates"] == tm["dates_total"] and 0 <= tm["filter_847"] <= tm["portfolio"]
        # top_n=10 under the 0.1 cap pins every weight at 0.1 (SLSQP lands within ~1e-10).  top_n=3 leaves
        # the weights free: SLSQP (ftol 1e-6) against the oracle's exact QP.
        np.testing.assert_allclose(v, np.asarray(r["portfolio"]["value"]), rtol=rtol, atol=0)
