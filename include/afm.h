/* afm.h -- C-ABI of the MI355X engine for the factor-research hot path of
 * Yuliang-Eliott/Alpha-Multi-factor-models.
 *
 * The reference has no FFI: its boundary is a set of pandas-in/pandas-out Python signatures
 * (SURVEY.md §8(b)).  Each entry point below replaces the compute behind one of them; the Python
 * mirror in alpha-multi-factor-models_amd/afm/ (ctypes) rebuilds the reference's DataFrames
 * around these calls, and INTEGRATION.md shows the binding a maintainer would add.
 *
 * Conventions
 *  - Every function returns 0 on success, a negative AFM_E* code on failure; the message of
 *    the last failure on the calling thread is afm_last_error().  Nothing throws across the ABI.
 *  - Buffers are caller-owned DEVICE pointers (hipMalloc / torch CUDA tensors) unless a
 *    parameter says "host".  The library never frees caller memory and keeps no global state
 *    besides the per-thread error string; work runs on the context's stream, asynchronously.
 *  - Panels are CALENDAR GRIDS: row-major [T][lda] float64 (date-major, asset-minor), lda a
 *    multiple of 64 >= A.  Presence of an asset-day is a bit mask: word [c][a] (uint64) holds
 *    days 64c..64c+63 of asset a in bits 0..63.  Windows are positional over each asset's
 *    present days, exactly as the reference's per-security pandas frames (No-talib.py:5-6).
 *  - Arithmetic is IEEE fp64 without FMA contraction, reproducing pandas 2.3.3 bit-for-bit.
 */
#ifndef AFM_H
#define AFM_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AFM_OK 0
#define AFM_E_ARG (-1)      /* invalid argument (shape, null pointer, alignment) */
#define AFM_E_HIP (-2)      /* HIP runtime error */
#define AFM_E_STATE (-3)    /* misuse (destroyed context, ...) */

typedef struct afm_ctx afm_ctx;

#define AFM_N_FACTORS 98    /* No-talib.py output columns: 96 factors + target + tmr_ret1d */

/* ---- context --------------------------------------------------------------------------- */
int afm_ctx_create(int device, afm_ctx** out);
/* stream: a hipStream_t (e.g. torch.cuda.current_stream().cuda_stream); NULL = default stream */
int afm_ctx_set_stream(afm_ctx* ctx, void* stream);
/* Execution options of a context -- work splits that never change a result (the invariance tests
 * set them; defaults are the library's choice):
 *   "factor_split"  0 (auto) | 1 | 3 | 5 | 15: workgroups per 64-asset block of the factor kernel
 *                   (the 15-set partition) | 103 | 105 | 106 | 110: 100 + workgroups per block
 *                   of the 30-set small-grid partition | 206: 6 workgroups per block of the
 *                   60-set partition (the N = 4 shard)
 *   "factor_pair"   1 (default) | 0: the 3-way split runs two items per workgroup
 *   "factor_fast"   1 (default) | 0: the clean-window fast step of the factor kernel
 *   "gram_checked"  0 (default) | 1: afm_xs_gram_f64 stages every row checked (no FAST + REDO) */
int afm_ctx_set_option(afm_ctx* ctx, const char* name, int64_t value);
/* The current value of an option of afm_ctx_set_option (value: out). */
int afm_ctx_get_option(afm_ctx* ctx, const char* name, int64_t* value);
/* A stream whose kernels run only on the compute units set in cu_mask (nwords 32-bit words, bit i
 * = the i-th compute unit of the device's logical CU mask; hipExtStreamCreateWithCUMask); the
 * pipeline places its FM per-date Grams on one so latency-bound kernels keep whole CUs.  *out:
 * the hipStream_t.  afm_stream_destroy releases it. */
int afm_stream_create_cu_mask(int device, const uint32_t* cu_mask, int nwords, void** out);
int afm_stream_destroy(void* stream);
int afm_ctx_destroy(afm_ctx* ctx);
const char* afm_last_error(void);
int afm_version(void);
/* Name of factor column i (0 <= i < AFM_N_FACTORS), No-talib.py creation order; host string. */
const char* afm_factor_name(int i);

/* ---- I0-I16: factor panel -- replaces compute_factors(data) (No-talib.py:1-93) -----------
 * Inputs [T][lda]: close_price, volume, ret1d, excess_ret1d; valid_bits [ceil(T/64)][lda].
 * out: [AFM_N_FACTORS][T][lda]; cells of absent asset-days hold NaN in the date rows the kernel
 * writes for their 64-asset block (a day with a present asset in the block), else untouched.
 * nanfree_bits [ceil(T/64)][lda]: present AND all 96 factor columns non-NaN (target/tmr_ret1d
 * excluded: their NaN-ness is read from their planes), i.e. the dropna() row mask of
 * No-talib.py:33 before the pass-through and label columns are considered.
 * finite_bits (optional, may be NULL): present AND all 96 factor columns finite (dropna keeps
 * +-inf, e.g. vol_change after a zero-volume day; the regression stages need finite rows).
 * ret1d and excess may both be NULL: the label planes 96-97 are then not written, and the caller
 * fills them with afm_labels_f64 (e.g. on another stream, or for another asset range). */
int afm_factors_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda,
                    const double* close, const double* volume, const double* ret1d,
                    const double* excess, const uint64_t* valid_bits,
                    double* out, uint64_t* nanfree_bits, uint64_t* finite_bits);
/* The same panel one TIME SLAB at a time (series longer than one GPU's HBM holds as output,
 * BASELINE config D): dates [t0, t1) of the [T]-date inputs, t0 a multiple of 64, called for
 * consecutive slabs from t0 = 0.  out [AFM_N_FACTORS][t1 - t0][lda], nanfree_bits / finite_bits
 * [ceil((t1 - t0)/64)][lda] hold the slab's dates only.  state: a device buffer of
 * afm_factors_state_bytes(ctx, A) bytes carrying every recurrence state and the observation
 * rings from one slab to the next; the concatenated slabs equal one afm_factors_f64 call bit for
 * bit. */
int64_t afm_factors_state_bytes(afm_ctx* ctx, int64_t A);
int afm_factors_slab_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0,
                         int64_t t1, const double* close, const double* volume,
                         const double* ret1d, const double* excess, const uint64_t* valid_bits,
                         double* out, uint64_t* nanfree_bits, uint64_t* finite_bits,
                         double* state);
/* The same slab written IN PLACE into the whole panel: out [AFM_N_FACTORS][T][lda] and the bit
 * words [ceil(T/64)][lda] of afm_factors_f64 receive the dates [t0, t1) (t0, and t1 unless it is
 * T, multiples of 64).  A pipeline can start on the first slab's dates (the z statistics of a
 * train window) while the next slab builds. */
int afm_factors_range_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0,
                          int64_t t1, const double* close, const double* volume,
                          const double* ret1d, const double* excess, const uint64_t* valid_bits,
                          double* out, uint64_t* nanfree_bits, uint64_t* finite_bits,
                          double* state);

/* afm_factors_range_f64 with the row masks left to the caller (no label planes): the factor
 * kernel's per-job-wave NaN / non-finite partial words go to part (afm_factors_part_words(ctx, A,
 * lda, t0, t1) uint64 words), and afm_factor_masks_f64 ORs them into the whole-panel
 * nanfree_bits / finite_bits words of [t0, t1) -- on any stream ordered after the slab, so a
 * pipeline runs the masks and what reads them beside the next slab.  The same execution options
 * (factor_split) for both calls. */
int64_t afm_factors_part_words(afm_ctx* ctx, int64_t A, int64_t lda, int64_t t0, int64_t t1);
int afm_factors_range_part_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0,
                               int64_t t1, const double* close, const double* volume,
                               const uint64_t* valid_bits, double* out, double* state,
                               uint64_t* part);
int afm_factor_masks_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0, int64_t t1,
                         const uint64_t* valid_bits, const uint64_t* part, uint64_t* nanfree_bits,
                         uint64_t* finite_bits);

/* out_bits = in_bits without each asset's last present day (valid_bits): the rows whose
 * shift(-1) labels are NaN.  Used to mask the regression rows up front (the Gram's REDO pass
 * would otherwise re-run those dates). */
int afm_drop_last_obs_bits(afm_ctx* ctx, int64_t T, int64_t lda, const uint64_t* valid_bits,
                           const uint64_t* in_bits, uint64_t* out_bits);
/* The same for the words of the dates [t0, t1) only (t0, and t1 unless it is T, multiples of
 * 64; each asset's last present day still from all T dates). */
int afm_drop_last_obs_bits_range(afm_ctx* ctx, int64_t T, int64_t lda, const uint64_t* valid_bits,
                                 const uint64_t* in_bits, uint64_t* out_bits, int64_t t0,
                                 int64_t t1);
/* target = excess_ret1d.shift(-1), tmr_ret1d = ret1d.shift(-1) per asset (No-talib.py:90-91) for
 * the grid dates [t0, t1) only (the label planes of afm_factors_f64 for a sub-range; used where
 * the factor panel itself is sharded by asset but the history/PnL planes are needed for every
 * asset).  Absent cells are not written. */
int afm_labels_f64(afm_ctx* ctx, int64_t T, int64_t lda, int64_t t0, int64_t t1,
                   const double* excess, const double* ret1d, const uint64_t* valid_bits,
                   double* target, double* tmr);

/* ---- R1: cross-sectional regression ---------------------------------------------------------
 * Segmented shifted Gram on fp64 MFMA.  Segment t (t = seg0 .. seg0+nseg-1) is the rows
 * [t*seg_stride, t*seg_stride + seg_rows) of every column; column c starts at base + c*col_stride.
 * Grid mode (bits != NULL): seg_stride = lda, seg_rows = A, segment = date t, a row is used when
 * bit (t & 63) of bits[(t >> 6) * lda + row] is set.  Long mode (bits == NULL): rows at or past
 * row_limit (>= 0) are masked.  Rows with any non-finite value among [x_cols.., y] are skipped.
 * Z = [1, x_cols[0..p), y]; gram[s] = sum (z - shift[s]) (z - shift[s])^T  ((p+2)^2 entries),
 * shift[s] = the first usable row (column 0 unshifted).  1 <= p <= 110.  cols: DEVICE int32[p]. */
int afm_xs_gram_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t seg_stride,
                    int64_t seg_rows, int64_t row_limit, const int32_t* cols, int p, int ycol,
                    const uint64_t* bits, int64_t seg0, int64_t nseg, double* gram, double* shift);
/* OLS with intercept per segment from (gram, shift): beta[s] = [intercept, b_1..b_p].  Scaled
 * (unit-diagonal) Cholesky of the centered normal equations; a regressor whose pivot falls below
 * tol is dropped (b = 0) -- rank[s] counts the kept ones.  Segments with n <= p get NaN. */
int afm_ols_solve_f64(afm_ctx* ctx, const double* gram, const double* shift, int p, int64_t nseg,
                      double tol, double* beta, double* nobs, int32_t* rank);
/* Exact (Chan) combination of nseg per-segment moments into one (gram, shift) -- the pooled OLS
 * of KKT:582-583 over the union of the segments' rows. */
int afm_pool_moments_f64(afm_ctx* ctx, const double* gram, const double* shift, int p,
                         int64_t nseg, double* out_gram, double* out_shift);
/* Segmented version: out[b] combines segments [b*per, min((b+1)*per, nseg)) in order (Chan), for
 * b < ceil(nseg/per) -- e.g. the per-rank partial moments of one date (multi-GPU asset shards), or
 * one level of afm_pool_moments_f64's tree.  Segments with n = 0 are skipped. */
int afm_pool_segments_f64(afm_ctx* ctx, const double* gram, const double* shift, int p,
                          int64_t nseg, int64_t per, double* out_gram, double* out_shift);
/* afm_pool_moments_f64's fixed tree (level 0 merges 16 segments, level 1 four level-0 results =
 * 64-date blocks, later levels 8 results each, until one remains) entered at level level0: the
 * multi-GPU step pools each rank's dates through levels 0-1 (afm_pool_segments_f64 with per 16,
 * then 4) and the gathered 64-date blocks with level0 = 2 -- the same tree as one device. */
int afm_pool_tree_f64(afm_ctx* ctx, const double* gram, const double* shift, int p, int64_t nseg,
                      int level0, double* out_gram, double* out_shift);
/* pred[t][a] = beta[t-t0][0] + sum_j beta[t-t0][1+j] * x_cols[j][t][a] on grid rows with a mask
 * bit (NaN elsewhere), t in [t0, t0+nt); beta_stride = 0 applies one coefficient vector.
 * ycheck >= 0: additionally require column ycheck finite (e.g. the label of a dropna'd row). */
int afm_predict_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda, int64_t t0,
                    int64_t nt, const int32_t* cols, int p, const double* beta,
                    int64_t beta_stride, const uint64_t* bits, int ycheck, double* pred);
/* Least-squares refinement helpers for a long design Z [..][n] (column j at Z + j*n):
 * r = (Z[ycol] - mean[p+1]) - sum_j beta[1+j] * (Z[j] - mean[1+j]) (mean = a pooled shift vector);
 * y += x; beta[0] = mean[p+1] - sum_j mean[1+j] * beta[1+j]. */
int afm_ols_residual_f64(afm_ctx* ctx, const double* Z, int64_t n, int p, int ycol,
                         const double* mean, const double* beta, double* r);
int afm_vec_add_f64(afm_ctx* ctx, int64_t n, const double* x, double* y);
int afm_ols_intercept_f64(afm_ctx* ctx, int p, const double* mean, double* beta);
/* Fama-MacBeth over segments with rank > 0: mean_t beta_t and mean / (std / sqrt(T)). */
int afm_fama_macbeth_f64(afm_ctx* ctx, const double* beta, const int32_t* rank, int64_t nseg,
                         int k, double* mean_out, double* t_out);
/* Lasso / elastic net by cyclic coordinate descent on centered moments -- replaces
 * sklearn Lasso(alpha=2e-4, max_iter=10000).fit (KKT:605-607; sklearn's
 * enet_coordinate_descent_gram, _cd_fast.pyx).  gram: ONE pooled shifted Gram [p+2][p+2] of
 * [1, x, y] (afm_pool_moments_f64), from which Q = X'X, q = X'y, y'y are centered in-kernel.
 * Minimises 0.5 ||y - X w||^2 + alpha_n ||w||_1 + 0.5 beta ||w||^2 (alpha_n = sklearn alpha * n)
 * from w = 0; stops when d_w_max / w_max < tol and the duality gap < tol * y'y, or at max_iter.
 * w[p] out; info[3] out = {gap, tol * y'y, n_iter}.  p <= 110. */
int afm_lasso_cd_f64(afm_ctx* ctx, const double* gram, int p, double alpha_n, double beta,
                     int max_iter, double tol, int positive, double* w, double* info);

/* ---- K1-K3: rebalance, weights, PnL -- replaces PortfolioManager (KKT:795-892) ---------------
 * Book arrays are [nd][2][AFM_MAX_BOOK] (long book, short book). */
#define AFM_MAX_BOOK 64
/* One call per set of rebalance dates (grid date indices `dates`, ascending, DEVICE int32[nd]).
 * pred [T][lda] (NaN = no prediction); trad_bits: present in all_df AND in_trading_universe=='Y';
 * hist/hist_bits: the history returns (df_train_y) and their presence; history rows are
 * [h_t0, h_t1) when window <= 0 (the reference: the whole training window), else the `window`
 * dates before each rebalance date; close/tmr: all_df close_price and tmr_ret1d.
 * Outputs: k_out[nd] (book size), books (asset indices, long descending / short ascending by
 * prediction, ties by ascending index), weights (exact min-variance, sum 1, lo <= w <= hi),
 * sums[nd][4] = {sum(tmr*w) long, short (numpy pairwise), sum(w*close) long, short (sequential)},
 * upos[nd][2][2][AFM_MAX_BOOK] / usize[nd][2]: members' positions in the id-union with the
 * previous / next date's prediction set (turnover alignment), status[nd] (0 ok, 1 QP cap,
 * 2 book larger than AFM_MAX_BOOK).  top_n <= AFM_MAX_BOOK. */
int afm_rebalance_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, const int32_t* dates,
                      int64_t nd, const double* pred, const uint64_t* trad_bits,
                      const double* hist, const uint64_t* hist_bits, int64_t h_t0, int64_t h_t1,
                      int64_t window, const double* close, const double* tmr, int top_n,
                      double lo, double hi, int32_t* k_out, int32_t* books, double* weights,
                      double* sums, int32_t* upos, int64_t* usize, int32_t* status);
/* Value / turnover recursion over the nd rebalance dates (KKT:864-892): value[nd+1] (value[0] =
 * v0), turnover[nd], long_ret[nd], short_ret[nd]. */
int afm_pnl_scan_f64(afm_ctx* ctx, int64_t nd, const int32_t* k_out, const int32_t* books,
                     const double* sums, const int32_t* upos, const int64_t* usize, double v0,
                     double rate, double* value, double* turnover, double* long_ret,
                     double* short_ret);
/* Bootstrap of the rebalance sequence (BASELINE config E): npaths paths of `steps` book slots
 * each, path [npaths][steps] (DEVICE int32, slots into the nd dates of one afm_rebalance_f64
 * call, drawn with replacement).  Every path re-runs the value / turnover recursion of
 * afm_pnl_scan_f64 (KKT:864-892) over its steps, with the turnover aligned on the union of the
 * previous and current step's prediction sets (pred [T][lda], dates as passed to
 * afm_rebalance_f64).  value [npaths][steps+1], turnover / long_ret / short_ret
 * [npaths][steps]. */
int afm_bootstrap_pnl_f64(afm_ctx* ctx, int64_t lda, const int32_t* dates, int64_t nd,
                          const double* pred, const int32_t* k_out, const int32_t* books,
                          const double* sums, int64_t npaths, int64_t steps, const int32_t* path,
                          double v0, double rate, double* value, double* turnover,
                          double* long_ret, double* short_ret);
/* determine_weights (KKT:817-833) for one book: R [rows][ld] returns (k columns, NaN = missing)
 * -> pairwise-complete covariance cov[k][k] and the exact box-QP weights w[k]. */
int afm_min_variance_weights_f64(afm_ctx* ctx, const double* R, int64_t rows, int64_t ld, int k,
                                 double lo, double hi, double* w, double* cov, int32_t* status);

/* ---- §8(f) rank 3: the talib factor variant (KKT:176-270) ------------------------------------
 * The 68 TA-Lib-defined columns for a calendar-grid panel (inputs as afm_factors_f64), out
 * [68][T][lda]: SMA_i 0-11, EMA_i 12-23, VSMA_i 24-35 (i = 6..50 step 4), BBANDS upper / middle /
 * lower 36-59 (i = 14..56 step 6), MACD_12_{18,24,30} 60-62, RSI_{8,14,20} 63-65, PVT 66, OBV 67
 * (TA-Lib 0.4 C-core semantics restated -- see csrc/talib.hip; the shared pandas columns come from
 * afm_factors_f64).  Absent cells are not written. */
int afm_talib_factors_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, const double* close,
                          const double* volume, const uint64_t* valid_bits, double* out);

/* ---- §8(f) rank 2: ingest / clean -- replaces merge_datasets' fill steps (KKT:113-166) ------
 * planes [K][T][lda] value columns on the union (date, id) grid, bits its presence words.
 * afm_ffill_f64: per security, NaN cells take the last non-NaN value of an earlier present date
 * (groupby('security_id') ... ffill(), KKT:145).
 * afm_date_mean_fill_f64: per date and column, NaN cells of present rows take the column mean
 * over the date's rows (pandas nanmean: numpy pairwise sum in security order with NaN -> 0, over
 * the non-NaN count; KKT:147).  scratch [K][T][lda].  A <= 65536.
 * afm_group_demean_f64: out = x - mean(x) per group of consecutive rows [offsets[g], offsets[g+1])
 * (Series.mean, numpy pairwise; excess_ret1d per date, KKT:154-161).  scratch [n]. */
int afm_ffill_f64(afm_ctx* ctx, int64_t K, int64_t T, int64_t lda, double* planes,
                  const uint64_t* bits);
int afm_date_mean_fill_f64(afm_ctx* ctx, int64_t K, int64_t T, int64_t A, int64_t lda,
                           double* planes, const uint64_t* bits, double* scratch);
int afm_group_demean_f64(afm_ctx* ctx, int64_t ngroups, const int64_t* offsets,
                         int64_t max_group, const double* x, double* out, double* scratch);

/* ---- A1-A4: signal evaluation -- replaces AlphaSignalAnalyzer.run (KKT:298-375) ----------
 * fr [3][T][lda]: k-th next present price row return c'/c - 1 for k = 1, 2, 5, NaN unless <= 1
 * (KKT:311-312); price_bits: presence of price_data rows. */
int afm_fwd_returns_f64(afm_ctx* ctx, int64_t T, int64_t lda, const double* close,
                        const uint64_t* price_bits, double* fr);
/* Per date: the merge/dropna cascade and per-date demeans of KKT:313-318 (numpy pairwise mean).
 * sig [T][lda] (NaN = no signal row).  Surviving rows, compacted in ascending asset order:
 * rows [4][T][lda] = {factor, return_1, return_2, return_5 (demeaned)}, rows_idx [T][lda] asset
 * index, nrows [T].  scratch [T][lda].  A <= 32768. */
int afm_xs_prepare_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, const double* sig,
                       const double* fr, double* scratch, double* rows, int32_t* rows_idx,
                       int32_t* nrows);
/* afm_xs_prepare_f64 on the dates [t0, t1) of the [T]-date buffers only (a rank's share of the
 * dates on N GPUs; T fixes the plane strides of fr and rows). */
int afm_xs_prepare_range_f64(afm_ctx* ctx, int64_t T, int64_t A, int64_t lda, int64_t t0,
                             int64_t t1, const double* sig, const double* fr, double* scratch,
                             double* rows, int32_t* rows_idx, int32_t* nrows);
/* Exact per-date ranks of the compacted factor column (method='first': ties by row order),
 * ascending and descending.  skey/sidx [T][lda] scratch. */
int afm_xs_rank_f64(afm_ctx* ctx, int64_t T, int64_t lda, const double* rows,
                    const int32_t* nrows, uint64_t* skey, int32_t* sidx, int32_t* rank_asc,
                    int32_t* rank_desc);
/* What afm_xs_stats_f64 reads of the ranks, without sorting (KKT:328-330, 359-369): rank_asc =
 * the first rank of the row's decile layer, rank_desc = the exact descending rank of the rows
 * ranked 1..10, nrows + 1 for the rest.  Same arguments as afm_xs_rank_f64 (lda > 12288: it). */
int afm_xs_layers_f64(afm_ctx* ctx, int64_t T, int64_t lda, const double* rows,
                      const int32_t* nrows, uint64_t* skey, int32_t* sidx, int32_t* rank_asc,
                      int32_t* rank_desc);
/* For the nd dates (DEVICE int32 grid indices): IC [nd][3] (nancorr Welford, KKT:344-345),
 * decile layer means [nd][3][10] and counts [nd][10] (KKT:328-332), top-10 factor-weighted
 * returns port [nd][3] (KKT:359-369; mcols = pivot columns present, <= 10). */
int afm_xs_stats_f64(afm_ctx* ctx, int64_t T, int64_t lda, const int32_t* dates, int64_t nd,
                     const double* rows, const int32_t* nrows, const int32_t* rank_asc,
                     const int32_t* rank_desc, int mcols, double* ic, double* layer_mean,
                     int32_t* layer_cnt, double* port);
/* Cumulative layers [nd][3][10], long-short [nd][3][5] (cum[10-l+1] - cum[l]), cumulative
 * top-10 returns [nd][3], IR [nyears][3] (year[nd] DEVICE int32, years year0..year0+nyears-1);
 * scratch [3*nyears][nd]. */
int afm_xs_series_f64(afm_ctx* ctx, int64_t nd, const double* layer_mean, const double* port,
                      const double* ic, const int32_t* year, int nyears, int year0,
                      double* cum_layer, double* ls, double* cum_port, double* ir,
                      double* scratch);

/* ---- per-security z-score -- replaces KKT:446-458 -----------------------
 * Column k of the K features is the plane base + cols[k] * col_stride ([T][lda], DEVICE int32
 * cols[K]); rows = grid cells with a set bit in bits [ceil(T/64)][lda] (the all_df rows).
 * Stats over the dates [t0, t1) (the train split): mu[k][lda] = groupby mean (Kahan),
 * sd[k][lda] = groupby std (Welford, ddof=1); NaN values are skipped, no rows -> NaN. */
int afm_zscore_stats_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t T,
                         int64_t lda, const int32_t* cols, int K, const uint64_t* bits,
                         int64_t t0, int64_t t1, double* mu, double* sd);
/* The same statistics streamed over consecutive date slabs [t0, t1) of one series (each slab at
 * least one date, the slabs in order): state [5][K][lda] doubles carries every (column, asset)
 * recurrence between the calls; first != 0 starts from zero, last != 0 writes mu / sd (else the
 * state is stored).  Bitwise the statistics of one afm_zscore_stats_f64 call over the union. */
int afm_zscore_stats_slab_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t T,
                              int64_t lda, const int32_t* cols, int K, const uint64_t* bits,
                              int64_t t0, int64_t t1, double* state, int first, int last,
                              double* mu, double* sd);
/* Over the rows of [t0, t1): z = (x - mu) / sd (IEEE), +-inf -> NaN, written to the plane
 * out + out_cols[k] * out_col_stride (out may alias base: in place when out_cols == cols);
 * other cells are not written.  keep [ceil(T/64)][lda]: the row bits of [t0, t1) with every z
 * non-NaN (the dropna() of KKT:449-451); every word of the chunks t0>>6 .. (t1-1)>>6 is
 * written, bits outside [t0, t1) cleared. */
int afm_zscore_apply_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t T,
                         int64_t lda, const int32_t* cols, int K, const uint64_t* bits,
                         int64_t t0, int64_t t1, const double* mu, const double* sd, double* out,
                         int64_t out_col_stride, const int32_t* out_cols, uint64_t* keep);

/* ---- the reference chain's regression on z-scored features (csrc/zgram.hip) ---------------
 * Replaces the z-scored design matrices of KKT:446-458 (never materialised: z is computed where
 * it is read) and the train+valid fit / test predict of KKT:582-612.
 * afm_zstats_finalize_f64: mu, sd [K][lda] (afm_zscore_stats_f64) -> zs [K+1][lda][2] =
 * {mu, 1/sd} (0, 0 where the column is unusable; row K = {0, 1}: identity for the regressand),
 * asset_ok[lda] = every column has a finite mean and sd > 0 (the assets that survive the z-score
 * dropna of KKT:452-454; every other asset has a NaN / inf z in all its rows). */
int afm_zstats_finalize_f64(afm_ctx* ctx, const double* mu, const double* sd, int K, int64_t lda,
                            double* zs, int32_t* asset_ok);
/* out[c][a] = a[c][a] & b[c][a] (b optional) & (asset_ok[a] ? ~0 : 0) (optional), restricted to
 * the dates [t0, t1): the split / dropna row sets on the calendar grid (KKT:426-458). */
int afm_row_bits(afm_ctx* ctx, int64_t nch, int64_t lda, const uint64_t* a, const uint64_t* b,
                 const int32_t* asset_ok, int64_t t0, int64_t t1, uint64_t* out);
/* Bytes of one partial Gram of afm_zgram_f64 / afm_zpool_f64 for p regressors (accumulator
 * layout: the upper-triangle 16 x 16 tile pairs of 2 tiles when p + 2 <= 32, else 7). */
int afm_zgram_part_bytes(int p);
/* Partial Grams of Z = [1, z_1..z_p, y] on fp64 MFMA (v_mfma_f64_16x16x4_f64), z_j = (x_j - mu)
 * * (1/sd) with {mu, 1/sd} = zs row zcols[j] (DEVICE int32; NULL = row j), y = plane ycol scaled
 * by zs row zid (the identity row of afm_zstats_finalize_f64); zs = NULL (afm_zgram_f64 only):
 * raw columns, no scaling; rows = set bits of `bits`;
 * regressor j is plane cols[j].  1 <= p <= 106; grid = workgroups (0: one per CU).
 * afm_zgram_f64 -- one partial per (date, asset block): dates [t0, t0+nt), block b = assets
 *   [blk0 + b*blk_assets, + blk_assets) below a_end; part [nt][nblk][part].  The per-date Grams
 *   of a regression on the cross-section (Fama-MacBeth).
 * afm_zpool_f64 -- one partial per (row-block r, date chunk c): the 64 assets [blk0 + 64r, +64)
 *   at every date of chunk c of [t0, t0+nt) (nchunk equal chunks); part [nrb][nchunk][part].
 *   The pooled Gram of every (date, asset) row (the design matrix of KKT:583 / 606): a
 *   workgroup keeps one row-block's {mu, 1/sd} in registers across its dates. */
int afm_zgram_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda,
                  const int32_t* cols, const int32_t* zcols, int p, int ycol, const double* zs,
                  int zid, const uint64_t* bits, int64_t t0, int64_t nt, int nblk, int64_t blk0,
                  int64_t blk_assets, int64_t a_end, double* part, int grid);
int afm_zpool_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda,
                  const int32_t* cols, const int32_t* zcols, int p, int ycol, const double* zs,
                  int zid, const uint64_t* bits, int64_t t0, int64_t nt, int64_t blk0, int nrb,
                  int64_t a_end, int nchunk, double* part, int grid);
/* Fixed-tree sum of partials: group g adds the leaves [g*per, min((g+1)*per, total)) (per <= 32)
 * over the binary tree of strides 1, 2, 4, 8, 16.  The tree composes -- a rank holding an aligned
 * power-of-two run of leaves computes one of its subtrees -- so every GPU count gets bit-identical
 * sums.  final_out: write symmetric Grams out[ngroups][p+2][p+2] (raw moments: entry [0][0] = n,
 * row 0 = column sums), else merged partials out[ngroups][part]. */
int afm_gram_tree_f64(afm_ctx* ctx, int p, const double* in, int64_t total, int per,
                      int final_out, double* out);
/* pred[t][a] = beta[0] + sum_j beta[1+j] * z_j (zero coefficients skipped), grid rows with a bit
 * set, t in [t0, t0+nt); NaN on the other cells of those dates.  (Lasso.predict, KKT:612.) */
int afm_zpredict_f64(afm_ctx* ctx, const double* base, int64_t col_stride, int64_t lda,
                     int64_t t0, int64_t nt, const int32_t* cols, int p, const double* zs,
                     const double* beta, const uint64_t* bits, double* pred);
/* Lasso(alpha, max_iter, tol).fit on one pooled (gram, shift) of [1, x, y] -- afm_lasso_cd_f64
 * with alpha_n = alpha * n read on the device, and beta_out[p+1] = [intercept, w] (sklearn's
 * _set_intercept: mean(y) - mean(x) . w).  info[3] = {gap, tol * y'y, n_iter}. */
int afm_lasso_fit_f64(afm_ctx* ctx, const double* gram, const double* shift, int p, double alpha,
                      int max_iter, double tol, int positive, double* beta_out, double* info);

#ifdef __cplusplus
}
#endif
#endif /* AFM_H */
