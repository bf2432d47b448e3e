"""ctypes binding of libafm.so (the C-ABI declared in include/afm.h).

The product path has no CPU fallback: if the library is missing or no GPU is visible, every
call raises.  ``make -C alpha-multi-factor-models_amd`` (or ``__graft_entry__.build()``) builds
the library in-tree.
"""
from __future__ import annotations

import ctypes
import os
import threading

HERE = os.path.dirname(os.path.abspath(__file__))
# AFM_LIB: an alternative build of the same library (A/B kernel variants, profiling builds)
LIB_PATH = os.environ.get("AFM_LIB") or os.path.join(HERE, "libafm.so")

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
DBL = ctypes.c_double

# name -> (restype, argtypes); kept in sync with include/afm.h (tests/test_abi.py checks it)
SIGNATURES = {
    "afm_ctx_create": (I32, [I32, ctypes.POINTER(P)]),
    "afm_ctx_set_stream": (I32, [P, P]),
    "afm_ctx_set_option": (I32, [P, ctypes.c_char_p, I64]),
    "afm_ctx_get_option": (I32, [P, ctypes.c_char_p, ctypes.POINTER(I64)]),
    "afm_stream_create_cu_mask": (I32, [I32, P, I32, ctypes.POINTER(P)]),
    "afm_stream_destroy": (I32, [P]),
    "afm_ctx_destroy": (I32, [P]),
    "afm_last_error": (ctypes.c_char_p, []),
    "afm_version": (I32, []),
    "afm_factor_name": (ctypes.c_char_p, [I32]),
    "afm_factors_f64": (I32, [P, I64, I64, I64, P, P, P, P, P, P, P, P]),
    "afm_factors_state_bytes": (I64, [P, I64]),
    "afm_factors_slab_f64": (I32, [P, I64, I64, I64, I64, I64, P, P, P, P, P, P, P, P, P]),
    "afm_factors_range_f64": (I32, [P, I64, I64, I64, I64, I64, P, P, P, P, P, P, P, P, P]),
    "afm_xs_gram_f64": (I32, [P, P, I64, I64, I64, I64, P, I32, I32, P, I64, I64, P, P]),
    "afm_ols_solve_f64": (I32, [P, P, P, I32, I64, DBL, P, P, P]),
    "afm_pool_moments_f64": (I32, [P, P, P, I32, I64, P, P]),
    "afm_pool_tree_f64": (I32, [P, P, P, I32, I64, I32, P, P]),
    "afm_pool_segments_f64": (I32, [P, P, P, I32, I64, I64, P, P]),
    "afm_labels_f64": (I32, [P, I64, I64, I64, I64, P, P, P, P, P]),
    "afm_drop_last_obs_bits": (I32, [P, I64, I64, P, P, P]),
    "afm_drop_last_obs_bits_range": (I32, [P, I64, I64, P, P, P, I64, I64]),
    "afm_factors_part_words": (I64, [P, I64, I64, I64, I64]),
    "afm_factors_range_part_f64": (I32, [P, I64, I64, I64, I64, I64, P, P, P, P, P, P]),
    "afm_factor_masks_f64": (I32, [P, I64, I64, I64, I64, I64, P, P, P, P]),
    "afm_predict_f64": (I32, [P, P, I64, I64, I64, I64, P, I32, P, I64, P, I32, P]),
    "afm_fama_macbeth_f64": (I32, [P, P, P, I64, I32, P, P]),
    "afm_ols_residual_f64": (I32, [P, P, I64, I32, I32, P, P, P]),
    "afm_vec_add_f64": (I32, [P, I64, P, P]),
    "afm_ols_intercept_f64": (I32, [P, I32, P, P]),
    "afm_lasso_cd_f64": (I32, [P, P, I32, DBL, DBL, I32, DBL, I32, P, P]),
    "afm_talib_factors_f64": (I32, [P, I64, I64, I64, P, P, P, P]),
    "afm_ffill_f64": (I32, [P, I64, I64, I64, P, P]),
    "afm_date_mean_fill_f64": (I32, [P, I64, I64, I64, I64, P, P, P]),
    "afm_group_demean_f64": (I32, [P, I64, P, I64, P, P, P]),
    "afm_rebalance_f64": (I32, [P, I64, I64, I64, P, I64, P, P, P, P, I64, I64, I64, P, P, I32,
                                DBL, DBL, P, P, P, P, P, P, P]),
    "afm_pnl_scan_f64": (I32, [P, I64, P, P, P, P, P, DBL, DBL, P, P, P, P]),
    "afm_bootstrap_pnl_f64": (I32, [P, I64, P, I64, P, P, P, P, I64, I64, P, DBL, DBL, P, P, P,
                                    P]),
    "afm_min_variance_weights_f64": (I32, [P, P, I64, I64, I32, DBL, DBL, P, P, P]),
    "afm_fwd_returns_f64": (I32, [P, I64, I64, P, P, P]),
    "afm_xs_prepare_f64": (I32, [P, I64, I64, I64, P, P, P, P, P, P]),
    "afm_xs_prepare_range_f64": (I32, [P, I64, I64, I64, I64, I64, P, P, P, P, P, P]),
    "afm_xs_rank_f64": (I32, [P, I64, I64, P, P, P, P, P, P]),
    "afm_xs_layers_f64": (I32, [P, I64, I64, P, P, P, P, P, P]),
    "afm_xs_stats_f64": (I32, [P, I64, I64, P, I64, P, P, P, P, I32, P, P, P, P]),
    "afm_xs_series_f64": (I32, [P, I64, P, P, P, P, I32, I32, P, P, P, P, P]),
    "afm_zscore_stats_f64": (I32, [P, P, I64, I64, I64, P, I32, P, I64, I64, P, P]),
    "afm_zscore_stats_slab_f64": (I32, [P, P, I64, I64, I64, P, I32, P, I64, I64, P, I32, I32,
                                        P, P]),
    "afm_zscore_apply_f64": (I32, [P, P, I64, I64, I64, P, I32, P, I64, I64, P, P, P, I64, P, P]),
    "afm_zgram_part_bytes": (I32, [I32]),
    "afm_zstats_finalize_f64": (I32, [P, P, P, I32, I64, P, P]),
    "afm_row_bits": (I32, [P, I64, I64, P, P, P, I64, I64, P]),
    "afm_zgram_f64": (I32, [P, P, I64, I64, P, P, I32, I32, P, I32, P, I64, I64, I32, I64, I64,
                            I64, P, I32]),
    "afm_zpool_f64": (I32, [P, P, I64, I64, P, P, I32, I32, P, I32, P, I64, I64, I64, I32, I64,
                            I32, P, I32]),
    "afm_gram_tree_f64": (I32, [P, I32, P, I64, I32, I32, P]),
    "afm_zpredict_f64": (I32, [P, P, I64, I64, I64, I64, P, I32, P, P, P, P]),
    "afm_lasso_fit_f64": (I32, [P, P, P, I32, DBL, I32, DBL, I32, P, P]),
}


class AfmError(RuntimeError):
    pass


_lib = None
_lock = threading.Lock()


def lib():
    global _lib
    if _lib is None:
        with _lock:
            if _lib is None:
                if not os.path.exists(LIB_PATH):
                    raise ImportError(f"{LIB_PATH} is not built: run `make -C "
                                      f"{os.path.dirname(HERE)}` (hipcc, gfx950)")
                L = ctypes.CDLL(LIB_PATH)
                for name, (res, args) in SIGNATURES.items():
                    f = getattr(L, name)
                    f.restype = res
                    f.argtypes = args
                _lib = L
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().afm_last_error().decode(errors="replace")
        raise AfmError(f"{what or 'afm'} failed ({rc}): {msg}")


class Context:
    """One afm_ctx per device; calls are issued on torch's current stream of that device."""

    _by_device: dict = {}

    def __init__(self, device: int):
        self.device = device
        h = P()
        check(lib().afm_ctx_create(device, ctypes.byref(h)), "afm_ctx_create")
        self.handle = h

    @classmethod
    def get(cls, device: int | None = None) -> "Context":
        import torch
        if not torch.cuda.is_available():
            raise AfmError("no GPU visible: the afm engine runs on MI355X only (no CPU fallback)")
        if device is None:
            device = torch.cuda.current_device()
        ctx = cls._by_device.get(device)
        if ctx is None:
            ctx = cls._by_device[device] = Context(device)
        return ctx

    def set_option(self, name: str, value: int):
        """afm_ctx_set_option: an execution option of this context (include/afm.h)."""
        check(lib().afm_ctx_set_option(self.handle, name.encode(), int(value)),
              f"afm_ctx_set_option({name})")

    def get_option(self, name: str) -> int:
        """afm_ctx_get_option: the current value of an execution option."""
        v = I64()
        check(lib().afm_ctx_get_option(self.handle, name.encode(), ctypes.byref(v)),
              f"afm_ctx_get_option({name})")
        return int(v.value)

    def bind_stream(self):
        import torch
        s = torch.cuda.current_stream(self.device).cuda_stream
        check(lib().afm_ctx_set_stream(self.handle, P(s)), "afm_ctx_set_stream")
        return self.handle


def ptr(t) -> P:
    """Device pointer of a contiguous torch tensor."""
    if not t.is_contiguous():
        raise AfmError("tensor must be contiguous")
    return P(t.data_ptr())


def factor_names() -> list:
    L = lib()
    return [L.afm_factor_name(i).decode() for i in range(98)]


class options:
    """Context manager: execution options of the device's context (afm_ctx_set_option) for the
    duration of a block, restored after it to the values they had before (nesting-safe) -- the
    invariance tests' work splits."""

    DEFAULTS = {"factor_split": 0, "factor_pair": 1, "factor_fast": 1, "gram_checked": 0}

    def __init__(self, device: int | None = None, **opts):
        self.device, self.opts = device, opts

    def __enter__(self):
        self.ctx = Context.get(self.device)
        self.saved = {k: self.ctx.get_option(k) for k in self.opts}
        for k, v in self.opts.items():
            self.ctx.set_option(k, v)
        return self.ctx

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            self.ctx.set_option(k, v)
        return False


def cu_mask_stream(device: int, exclude: int):
    """A torch stream on ``device`` whose kernels avoid ``exclude`` compute units (spread evenly
    over the logical CU mask), made by afm_stream_create_cu_mask; the pipeline's FM side stream
    (PipelineConfig.fm_free_cus).  The stream lives as long as the returned object."""
    import torch
    n = torch.cuda.get_device_properties(device).multi_processor_count
    if not 0 < exclude < n:
        raise AfmError(f"exclude must be in 1..{n - 1} compute units")
    keep = [True] * n
    for i in range(exclude):                       # every (n / exclude)-th CU left free
        keep[(i * n) // exclude] = False
    words = (ctypes.c_uint32 * ((n + 31) // 32))()
    for i, k in enumerate(keep):
        if k:
            words[i // 32] |= 1 << (i % 32)
    h = P()
    check(lib().afm_stream_create_cu_mask(device, words, len(words), ctypes.byref(h)),
          "afm_stream_create_cu_mask")
    return _MaskedStream(device, h)


class _MaskedStream:
    def __init__(self, device, handle):
        import torch
        self.handle = handle
        self.stream = torch.cuda.ExternalStream(handle.value, device=torch.device("cuda", device))

    def __del__(self):
        try:
            lib().afm_stream_destroy(self.handle)
        except Exception:
            pass
