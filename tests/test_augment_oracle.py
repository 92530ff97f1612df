"""CPU checks of the training-sample transform: the C oracle against the
Pillow goldens (bit exact), the host-side mirror (crop spec parsing, the seeded jitter draws,
the resample plan computed by the C-ABI library) against the reference / the oracle.
No GPU: the HIP kernels are checked in tests/test_augment.py (-m gpu)."""
import ctypes
import hashlib
import random

import numpy as np
import pytest

import golden_util as gu
from oracle import augment_oracle as A

Z = np.load(gu.GOLDEN_DIR + "/augment_pil.npz")


def test_oracle_resize_matches_pillow():
    for i in range(int(Z["n_resize"])):
        img, box, out = Z[f"resize{i}_in"], tuple(int(v) for v in Z[f"resize{i}_box"]), Z[f"resize{i}_out"]
        got = A.resize(A.crop(img, box), *out.shape[:2])
        np.testing.assert_array_equal(got, out, err_msg=f"resize case {i}")


def test_oracle_resize_kitti_size():
    kin = np.random.default_rng(7).integers(0, 256, (375, 1242, 3), dtype=np.uint8)
    assert hashlib.sha256(kin.tobytes()).digest() == Z["kitti_in_sha"].tobytes(), "input generator drifted"
    out = A.resize(kin, 192, 640)
    np.testing.assert_array_equal(out[[0, 1, 95, 190, 191]], Z["kitti_out_rows"])
    assert hashlib.sha256(out.tobytes()).digest() == Z["kitti_out_sha"].tobytes()


def _golden_jitter(k):
    if not bool(Z[f"jit{k}_apply"]):
        return A.make_jitter(apply=0)
    f, order, m = Z[f"jit{k}_f"], [int(v) for v in Z[f"jit{k}_order"]], Z[f"jit{k}_m"]
    return A.make_jitter(order=order, factors=f[:3], hue_shift=int(np.array(f[3] * 255).astype(np.uint8)),
                         matrix=None if np.isnan(m).any() else m)


def test_oracle_jitter_matches_pillow():
    img = Z["jitter_img"]
    for k in range(int(Z["n_jit"])):
        np.testing.assert_array_equal(A.color_jitter(img, _golden_jitter(k)), Z[f"jit{k}_out"], err_msg=f"jitter {k}")


def test_oracle_hue_exhaustive():
    """adjust_hue over all 2^24 colours, against Pillow's result (sha256 pinned)."""
    allc = np.arange(1 << 24, dtype=np.uint32)
    every = np.stack([(allc >> 16) & 255, (allc >> 8) & 255, allc & 255], -1).astype(np.uint8).reshape(4096, 4096, 3)
    for shift in (0, 7, 244):
        out = A.color_jitter(every, A.make_jitter(order=(3, 0, 1, 2), hue_shift=shift))
        assert hashlib.sha256(out.tobytes()).digest() == Z[f"hue_all_{shift}"].tobytes(), shift


def test_oracle_full_sample():
    box = tuple(int(v) for v in Z["sample_box"])
    from packnet_sfm_amd.datasets.augmentations import random_color_jitter_params
    d = random_color_jitter_params((0.2, 0.2, 0.2, 0.05), 1.0, random.Random(int(Z["sample_seed"])))
    j = A.make_jitter(order=d["order"], factors=d["factors"], hue_shift=d["hue_shift"], matrix=d["matrix"])
    orig, rgb = A.train_transform(list(Z["sample_in"]), box, (24, 80), j)
    for i in range(3):
        np.testing.assert_array_equal(orig[i], Z["sample_orig"][i].transpose(2, 0, 1) / np.float32(255))
        np.testing.assert_array_equal(rgb[i], Z["sample_rgb"][i].transpose(2, 0, 1) / np.float32(255))


def test_jitter_draws_follow_reference_order():
    from packnet_sfm_amd.datasets.augmentations import random_color_jitter_params
    for k in range(int(Z["n_jit"])):
        par = tuple(float(v) for v in Z[f"jit{k}_params"])
        par = par[:4] if par[4] == 0 else par
        d = random_color_jitter_params(par, float(Z[f"jit{k}_prob"]), random.Random(int(Z[f"jit{k}_seed"])))
        assert d["apply"] == bool(Z[f"jit{k}_apply"])
        if d["apply"]:
            assert d["factors"] + [d["hue_factor"]] == list(Z[f"jit{k}_f"])
            assert d["order"] == list(Z[f"jit{k}_order"])
            assert d["hue_shift"] == int(np.array(d["hue_factor"] * 255).astype(np.uint8))
            m = Z[f"jit{k}_m"]
            assert (d["matrix"] is None) == bool(np.isnan(m).any())
            if d["matrix"] is not None:
                assert d["matrix"] == list(m)


def test_parse_crop_borders_matches_reference():
    from packnet_sfm_amd.utils.misc import parse_crop_borders
    for i in range(int(Z["n_crop"])):
        n = int(Z[f"crop{i}_len"])
        spec = tuple(int(v) if isint else float(v)
                     for v, isint in zip(Z[f"crop{i}_spec"][:n], Z[f"crop{i}_isint"][:n]))
        shape = tuple(int(v) for v in Z[f"crop{i}_shape"])
        assert parse_crop_borders(spec, shape) == tuple(int(v) for v in Z[f"crop{i}_box"]), spec


@pytest.fixture(scope="module")
def hip():
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd import _hip
    return _hip


@pytest.mark.parametrize("src,box,out", [((375, 1242), (13, 23, 1229, 375), (192, 640)),
                                         ((375, 1242), (0, 0, 1242, 375), (192, 640)),
                                         ((24, 80), (0, 0, 80, 24), (48, 160)),
                                         ((61, 40), (0, 0, 40, 61), (30, 40)),
                                         ((50, 90), (-7, 5, 80, 58), (20, 33)),
                                         ((1216, 1936), (0, 0, 1936, 1216), (384, 640))])
def test_plan_matches_oracle(hip, src, box, out):
    """psfm_augment_plan (host code of the C-ABI library) == Pillow's precompute_coeffs."""
    p = hip.AugmentParams(n_samples=1, n_img=1, src_h=src[0], src_w=src[1], src_stride=src[0] * src[1] * 3,
                          crop_l=box[0], crop_t=box[1], crop_r=box[2], crop_b=box[3], out_h=out[0], out_w=out[1])
    L = hip.lib()
    n = L.psfm_augment_plan(ctypes.byref(p), None)
    plan = np.zeros(n, np.int32)
    assert L.psfm_augment_plan(ctypes.byref(p), plan.ctypes.data_as(ctypes.c_void_p)) == n
    kh, kv, rows, obh, och, obv, ocv, y0 = (int(v) for v in plan[:8])
    cw, ch = box[2] - box[0], box[3] - box[1]
    for (ins, outs, k, ob, oc, shift, tap_major) in ((cw, out[1], kh, obh, och, 0, False),
                                                     (ch, out[0], kv, obv, ocv, y0, False)):
        if ins == outs:
            assert k == 1
            continue
        k2, b, c = A.resample_plan(ins, outs)
        assert k == k2
        bb = plan[ob:ob + 2 * outs].reshape(outs, 2).copy()
        bb[:, 0] += shift
        np.testing.assert_array_equal(bb, b)
        cc = plan[oc:oc + k * outs].reshape(k, outs).T if tap_major else plan[oc:oc + k * outs].reshape(outs, k)
        np.testing.assert_array_equal(cc, c)
    assert hip.lib().psfm_augment_ws_bytes(ctypes.byref(p)) > 0


def test_abi_rejects_bad_arguments(hip):
    L = hip.lib()
    p = hip.AugmentParams(n_samples=2, n_img=3, src_h=10, src_w=10, src_stride=300, crop_l=0, crop_t=0, crop_r=10,
                          crop_b=10, out_h=5, out_w=5)
    dummy = ctypes.c_void_p(16)
    rc = L.psfm_train_augment(ctypes.byref(p), dummy, dummy, dummy, dummy, dummy, None, None)
    assert rc != 0 and b"multiple" in L.psfm_augment_last_error()
    p.n_img, p.crop_r = 4, 0
    assert L.psfm_augment_plan(ctypes.byref(p), None) < 0
    assert b"crop" in L.psfm_augment_last_error()
