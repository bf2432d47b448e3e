"""Can the FM per-date Grams run beside the z statistics instead of in the step's tail?  Times,
on a config-C step's buffers: the z statistics alone, the FM partial Grams (over the all_df
finite rows, frows -- available right after the factor kernel) alone, both on two streams at
once, and the FM Grams on a CU-masked stream (keeping K CUs) beside the z statistics.
    python tools/fm_overlap_probe.py [--assets 10000]"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "alpha-multi-factor-models_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--assets", type=int, default=10000)
    ap.add_argument("--reps", type=int, default=3)
    a = ap.parse_args()
    import torch
    import afm
    from afm import _lib
    from afm.factors import TARGET
    from afm.pipeline import Pipeline, PipelineConfig
    from afm.synthetic import make_panel
    grid = afm.PanelGrid.from_panel(make_panel(a.assets, 5040, seed=2023, tradable_p=0.9))
    pipe = Pipeline(grid, PipelineConfig())
    pipe.step()
    torch.cuda.synchronize()
    L, P, chk = _lib.lib(), _lib.ptr, _lib.check
    ctx = _lib.Context.get(0)
    T, lda, p, pf = pipe.T, pipe.lda_r, pipe.p, pipe.pf
    ncu = torch.cuda.get_device_properties(0).multi_processor_count

    def zstats():
        h = ctx.bind_stream()
        chk(L.afm_zscore_stats_f64(h, P(pipe.out), T * lda, T, lda, P(pipe.feat), p, P(pipe.alldf),
                                   0, pipe.sp.tr1, P(pipe.mu), P(pipe.sd)), "zstats")

    def fm(grid_wgs=0):
        h = ctx.bind_stream()
        chk(L.afm_zgram_f64(h, P(pipe.out), T * lda, lda, P(pipe.fm_cols), None, pf, TARGET, None,
                            0, P(pipe.frows), 0, T, pipe.nblk_r, 0, pipe.blk, pipe.A_r,
                            P(pipe.fm_part), grid_wgs), "fm")

    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    masked = {k: _lib.cu_mask_stream(0, ncu - k) for k in (32, 64, 96)}

    def timed(fn):
        ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
        best = 1e9
        for _ in range(a.reps):
            torch.cuda.synchronize()
            ev[0].record()
            fn()
            cur = torch.cuda.current_stream()
            for s in [s1, s2] + [m.stream for m in masked.values()]:
                cur.wait_stream(s)
            ev[1].record()
            torch.cuda.synchronize()
            best = min(best, ev[0].elapsed_time(ev[1]))
        return best

    def both(fm_stream, wgs):
        cur = torch.cuda.current_stream()
        s1.wait_stream(cur)
        fm_stream.wait_stream(cur)
        with torch.cuda.stream(s1):
            zstats()
        with torch.cuda.stream(fm_stream):
            fm(wgs)
    print(f"zstats alone {timed(zstats):.3f} ms", flush=True)
    print(f"fm alone {timed(fm):.3f} ms", flush=True)
    print(f"zstats + fm, two streams {timed(lambda: both(s2, 0)):.3f} ms", flush=True)
    def fm_on(stream, wgs):
        stream.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(stream):
            fm(wgs)
    for k, m in masked.items():
        print(f"fm alone on {k} CUs {timed(lambda: fm_on(m.stream, k)):.3f} ms", flush=True)
        print(f"zstats + fm on {k} CUs {timed(lambda: both(m.stream, k)):.3f} ms", flush=True)


if __name__ == "__main__":
    main()
