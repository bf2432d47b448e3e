"""afm -- MI355X-native engine for the factor-research hot path of
Yuliang-Eliott/Alpha-Multi-factor-models.

Drop-in Python surface (same names, arguments and results as the reference):

* ``compute_factors(data)``                      -- No-talib.py:1-93
* ``AlphaSignalAnalyzer(df, name, prices).run()`` -- KKT Yuliang Jiang.py:280-375
* ``LinearRegression().fit/predict``              -- KKT:582-598 (pooled OLS)
* ``Lasso(alpha, max_iter).fit/predict``           -- KKT:605-607 (coordinate descent)
* ``PortfolioManager(...)``                       -- KKT:795-970
* ``split_zscore(all_df)``                       -- KKT:424-458 (z-score + split)

All compute runs in hand-written HIP kernels (libafm.so, C-ABI in include/afm.h); there is no
CPU fallback.
"""
from .factors import FACTOR_NAMES, compute_factors, factor_panel  # noqa: F401
from .grid import PanelGrid, pack_bits, unpack_bits  # noqa: F401
from . import regression  # noqa: F401
from .regression import Lasso, LinearRegression, cross_sectional_ols  # noqa: F401
from .analyzer import AlphaSignalAnalyzer  # noqa: F401
from .portfolio import PortfolioManager  # noqa: F401
from .zscore import split_zscore, zscore_grid  # noqa: F401

__all__ = ["compute_factors", "factor_panel", "FACTOR_NAMES", "PanelGrid", "pack_bits",
           "unpack_bits", "LinearRegression", "Lasso", "cross_sectional_ols", "AlphaSignalAnalyzer",
           "PortfolioManager", "split_zscore", "zscore_grid"]
