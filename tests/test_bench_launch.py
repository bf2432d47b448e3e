"""bench.py's multi-rank harness (the driver's N > 1 runs).

CPU: the --gpus / WORLD_SIZE rule (a bare ``--gpus N`` self-launches N ranks; under a launcher
--gpus must equal WORLD_SIZE), checked before anything imports torch.
GPU: ``bench.py --gpus 2`` started bare spawns ``torch.distributed.run`` as a child, the two ranks
(gloo, sharing cuda:0) run the timed steps behind the barrier / max-over-ranks clock, rank 0's one
JSON line comes back through the parent -- and its final portfolio value equals the one-GPU run's.
"""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")
SMALL = ["--assets", "1000", "--days", "640", "--steps", "2", "--warmup", "1",
         "--train-end", "2001-06-29", "--valid-end", "2001-12-31", "--window", "120",
         "--no-variants", "--no-configs", "--no-cpu-baseline"]


def _bench_module():
    sys.path.insert(0, ROOT)
    import importlib
    return importlib.import_module("bench")


def test_launch_world_rule(monkeypatch):
    b = _bench_module()
    monkeypatch.delenv("WORLD_SIZE", raising=False)
    assert b.launch_world(None) == (1, False)
    assert b.launch_world(1) == (1, False)
    assert b.launch_world(8) == (8, True)
    with pytest.raises(SystemExit):
        b.launch_world(0)
    monkeypatch.setenv("WORLD_SIZE", "4")
    assert b.launch_world(None) == (4, False)
    assert b.launch_world(4) == (4, False)
    with pytest.raises(SystemExit):
        b.launch_world(2)


def test_mismatched_gpus_under_launcher_exits_before_torch():
    env = dict(os.environ, WORLD_SIZE="2", RANK="0", LOCAL_RANK="0")
    r = subprocess.run([sys.executable, BENCH, "--gpus", "4"], env=env, capture_output=True,
                       text=True, timeout=60)
    assert r.returncode != 0 and "WORLD_SIZE=2" in r.stderr


def _run(gpus):
    env = dict(os.environ, AFM_BENCH_BACKEND="gloo")
    r = subprocess.run([sys.executable, "-u", BENCH, "--gpus", str(gpus)] + SMALL, cwd=ROOT,
                       env=env, capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [s for s in r.stdout.splitlines() if s.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0]), r.stderr


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_self_launch_two_ranks():
    d2, err = _run(2)
    assert "launching 2 ranks" in err
    assert d2["n_gpus"] == 2 and d2["steps"] == 2 and d2["warmup"] == 1
    assert d2["ms_per_step"] > 0 and d2["value"] > 0
    assert "exchange" in d2["stage_ms"]
    d1, _ = _run(1)
    assert d1["n_gpus"] == 1
    assert d1["config"]["asset_days"] == d2["config"]["asset_days"]
    # the sharded step is bit-identical to the one-device step (tests/test_sharded.py)
    assert d2["final_value"] == d1["final_value"]
    # one GPU: the rooflines divide by the kernel's own event time where the step path records
    # it (the pooled Gram's partial kernel always; this small grid builds its factor panel in
    # time slabs, so the factor roofline keeps its stage time), never more than the stage's
    roofs = {r["bound"]: r for r in (d1["roofline"], d1["roofline_next"])}
    for r in roofs.values():
        assert 0 < r["kernel_ms"] <= r["stage_ms"]
        assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=1e-2)
    assert roofs["hbm"]["kernel"].startswith("factor_panel_kernel")
    assert roofs["mfma"]["kernel"].startswith("zgram_kernel<7,1> (pooled")
    assert roofs["mfma"]["kernel_ms"] < roofs["mfma"]["stage_ms"]


@pytest.mark.gpu
@pytest.mark.timeout(600)
def test_bench_line_contract():
    """One GPU, a small panel, with the CPU-baseline leg: the one JSON line carries every key of
    the bench contract (metric / value / unit / n_gpus / steps / warmup / ms_per_step /
    higher_is_better / scaling / vs_baseline / dtype / data / config) plus the roofline and
    cpu_baseline objects, with consistent numbers."""
    env = dict(os.environ)
    args = [a for a in SMALL if a != "--no-cpu-baseline"]
    r = subprocess.run([sys.executable, "-u", BENCH] + args, cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=540)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [s for s in r.stdout.splitlines() if s.strip()]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step",
              "higher_is_better", "scaling", "vs_baseline", "dtype", "data", "config",
              "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1
    assert d["higher_is_better"] is True and d["scaling"] == "strong" and d["dtype"] == "f64"
    assert d["unit"] == "asset-days/s" and d["vs_baseline"] is None
    assert "workload" in d["config"] and "model" not in d["config"]
    # value = the whole panel's asset-days over the measured step time
    assert d["value"] == pytest.approx(d["config"]["asset_days"] / (d["ms_per_step"] * 1e-3),
                                       rel=1e-3)
    rf = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in rf, k
    assert rf["bound"] in ("hbm", "mfma") and 0 < rf["frac"] < 1
    cb = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in cb, k
    assert cb["value"] > 0 and cb["cores"] == 1 and cb["kind"] in ("port", "reference")

