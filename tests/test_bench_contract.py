"""bench.py's reporting logic on CPU (no GPU work): the roofline's stamped PMC profile is attached
only when it was taken on the current library sources and the same workload."""
import json

import bench


def test_stale_or_foreign_pmc_profile_is_not_attached(tmp_path, monkeypatch):
    args = bench.parse(["--config", "kitti-resnet-san"])
    key = bench.config_key(args)
    d = tmp_path / "profiles" / "pmc"
    d.mkdir(parents=True)
    monkeypatch.setattr(bench, "ROOT", str(tmp_path))
    monkeypatch.setattr(bench, "source_hash", lambda: "current0000000000")
    prof = {"config_key": key, "source_hash": "current0000000000",
            "kernels": {"K12_photometric_fwd_grad": {"hbm_bytes": 7.1e7, "SQ_ACTIVE_INST_VALU": 1e7}}}
    (d / f"{key}.json").write_text(json.dumps(prof))
    got, _, why = bench.stamped_profile(args)
    assert got is not None and why is None
    ktimes = {"K12_photometric_fwd_grad": 100.0, "prepass": 12.0}
    r = bench.roofline(args, ktimes)
    assert r["traffic"] == int(7.1e7)
    # the kernel's distance from its own VALU issue floor, beside the HBM fraction
    v = r["valu"]
    assert abs(v["valu_floor_us_over_dominant_us"] - v["simd_floor_us_2cyc"] / r["dominant_us_per_launch"]) < 2e-3
    prof["source_hash"] = "older00000000000"
    (d / f"{key}.json").write_text(json.dumps(prof))
    got, _, why = bench.stamped_profile(args)
    assert got is None and why.startswith("stale")
    r = bench.roofline(args, ktimes)
    assert r["traffic"] is None and "stale" in r["profile"]
    prof.update(source_hash="current0000000000", config_key="other")
    (d / f"{key}.json").write_text(json.dumps(prof))
    assert bench.stamped_profile(args)[0] is None


def test_algorithmic_bytes_follow_survey():
    # 120 B/px at N=2, S=4 -> 14,745,600 B per 192x640 image
    assert bench.algorithmic_bytes_per_image(192, 640) == 14_745_600


def test_committed_bench_lines_keep_the_contract():
    """The committed bench lines (profiles/r04/final) carry the driver's JSON contract: the headline
    keys, the roofline object (dominant kernel against HBM, timed in the step) and, for the default
    config, the CPU baseline object."""
    import glob
    import json
    import os
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    files = sorted(f for r in ("r04", "r06") for f in glob.glob(os.path.join(root, "profiles", r, "final", "bench_*.json"))
                   if "rehearsal" not in f)   # the N = 2 gloo rehearsal runs without the kernel timing
    assert files
    for f in files:
        d = json.loads(open(f).read().strip().splitlines()[-1])
        for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
                  "scaling", "vs_baseline", "dtype", "data", "config", "roofline"):
            assert k in d, (f, k)
        assert d["n_gpus"] >= 1 and d["higher_is_better"] is True and d["value"] > 0
        r = d["roofline"]
        for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
            assert k in r, (f, k)
        assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
        assert "workload" in d["config"]
        if f.endswith("bench_kitti-resnet-san.json") and "r04" in f or "bench_default" in f:
            cb = d["cpu_baseline"]
            for k in ("value", "unit", "cores", "kind", "sample"):
                assert k in cb, k
        if "r06" in f and "bench_default" in f:   # the stamped profile of its own sources was attached
            assert r["traffic"] and r["valu"]["valu_floor_us_over_dominant_us"] > 0
