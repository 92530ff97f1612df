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
    assert bench.roofline(args, ktimes)["traffic"] == int(7.1e7)
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
