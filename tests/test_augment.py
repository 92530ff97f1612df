"""GPU parity of the training-sample transform (include/psfm_augment.h):
the HIP kernels against the Pillow goldens and the C oracle — bit exact (byte / integer work;
fp32 outputs are u8 / 255 exactly)."""
import hashlib
import random

import numpy as np
import pytest
import torch

import golden_util as gu
from oracle import augment_oracle as A

pytestmark = pytest.mark.gpu
Z = np.load(gu.GOLDEN_DIR + "/augment_pil.npz")
DEV = "cuda:0"


@pytest.fixture(scope="module")
def aug():
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.datasets import augmentations
    return augmentations


def chw(u8_hwc):
    return torch.from_numpy(np.ascontiguousarray(u8_hwc.transpose(2, 0, 1))).float() / 255


def to_u8(t):
    """fp32 u / 255 -> u (exact inverse for u8 inputs)."""
    return (t.cpu() * 255).round().to(torch.uint8)


def oracle_jitter(d):
    if not d["apply"]:
        return A.make_jitter(apply=0)
    return A.make_jitter(order=d["order"], factors=d["factors"], hue_shift=d["hue_shift"], matrix=d["matrix"])


def test_resize_goldens(aug):
    for i in range(int(Z["n_resize"])):
        img, box, out = Z[f"resize{i}_in"], tuple(int(v) for v in Z[f"resize{i}_box"]), Z[f"resize{i}_out"]
        orig, rgb = aug.augment_images(torch.from_numpy(img)[None].to(DEV), 1, box, out.shape[:2])
        assert rgb is None
        torch.testing.assert_close(orig[0].cpu(), chw(out), rtol=0, atol=0, msg=f"resize case {i}")


def test_kitti_resize_golden(aug):
    kin = np.random.default_rng(7).integers(0, 256, (375, 1242, 3), dtype=np.uint8)
    orig, _ = aug.augment_images(torch.from_numpy(kin)[None].to(DEV), 1, (0, 0, 1242, 375), (192, 640))
    u8 = to_u8(orig[0]).permute(1, 2, 0).contiguous().numpy()
    np.testing.assert_array_equal(u8[[0, 1, 95, 190, 191]], Z["kitti_out_rows"])
    assert hashlib.sha256(u8.tobytes()).digest() == Z["kitti_out_sha"].tobytes()


def test_jitter_goldens(aug):
    img = Z["jitter_img"]
    h, w = img.shape[:2]
    for k in range(int(Z["n_jit"])):
        par = tuple(float(v) for v in Z[f"jit{k}_params"])
        par = par[:4] if par[4] == 0 else par
        d = aug.random_color_jitter_params(par, float(Z[f"jit{k}_prob"]), random.Random(int(Z[f"jit{k}_seed"])))
        orig, rgb = aug.augment_images(torch.from_numpy(img)[None].to(DEV), 1, (0, 0, w, h), (h, w), [d])
        torch.testing.assert_close(orig[0].cpu(), chw(img), rtol=0, atol=0)
        torch.testing.assert_close(rgb[0].cpu(), chw(Z[f"jit{k}_out"]), rtol=0, atol=0, msg=f"jitter {k}")


def test_hue_exhaustive(aug):
    """Every RGB colour through adjust_hue on the GPU == Pillow (sha256 pinned)."""
    allc = torch.arange(1 << 24, dtype=torch.int64)
    every = torch.stack([(allc >> 16) & 255, (allc >> 8) & 255, allc & 255], -1).to(torch.uint8).view(1, 4096, 4096, 3)
    every = every.to(DEV)
    for shift in (0, 7, 244):
        d = dict(apply=True, order=[3, 0, 1, 2], factors=[1.0, 1.0, 1.0], hue_factor=0.0, hue_shift=shift, matrix=None)
        _, rgb = aug.augment_images(every, 1, (0, 0, 4096, 4096), (4096, 4096), [d])
        u8 = to_u8(rgb[0]).permute(1, 2, 0).contiguous().numpy()
        assert hashlib.sha256(u8.tobytes()).digest() == Z[f"hue_all_{shift}"].tobytes(), shift
        del rgb


def test_full_sample_golden(aug):
    box = tuple(int(v) for v in Z["sample_box"])
    imgs = torch.from_numpy(Z["sample_in"]).to(DEV)          # [3, h, w, 3]: rgb + 2 contexts, B = 1
    d = aug.random_color_jitter_params((0.2, 0.2, 0.2, 0.05), 1.0, random.Random(int(Z["sample_seed"])))
    orig, rgb = aug.augment_images(imgs, 1, box, (24, 80), [d])
    for i in range(3):
        torch.testing.assert_close(orig[i].cpu(), chw(Z["sample_orig"][i]), rtol=0, atol=0)
        torch.testing.assert_close(rgb[i].cpu(), chw(Z["sample_rgb"][i]), rtol=0, atol=0)


@pytest.mark.parametrize("src,borders,shape,jit,B,N", [
    ((375, 1242), (-352, 0, 0.5, 1216), (192, 640), (0.2, 0.2, 0.2, 0.05), 4, 2),   # tiny config + KITTI resize
    ((375, 1242), (), (192, 640), (0.2, 0.2, 0.2, 0.05, 0.1), 2, 2),                # full frame, colour matrix
    ((370, 1224), (-352, 0, 0.5, 1216), (), (0.5, 0.5, 0.5, 0.2), 2, 1),            # crop only (no resize)
    ((48, 160), (), (96, 320), (0.2, 0.2, 0.2, 0.05), 3, 2),                        # upscale
    ((64, 200), (), (64, 200), (), 2, 2),                                            # identity, no jitter
    ((1216, 1936), (), (384, 640), (0.2, 0.2, 0.2, 0.05), 1, 2),                     # DDAD: 21-tap generic paths
])
def test_batch_matches_oracle(aug, src, borders, shape, jit, B, N):
    g = np.random.default_rng(hash((src, shape, B)) & 0xffff)
    n_img = B * (1 + N)
    imgs = g.integers(0, 256, (n_img,) + src + (3,), dtype=np.uint8)
    batch = {"rgb": torch.from_numpy(imgs[:B]).to(DEV),
             "rgb_context": [torch.from_numpy(imgs[(j + 1) * B:(j + 2) * B]).to(DEV) for j in range(N)],
             "intrinsics": torch.tensor([[721.5, 0, 609.6], [0, 721.5, 172.9], [0, 0, 1]]).repeat(B, 1, 1)}
    out = aug.train_transforms_batch(batch, shape, jit, borders, prob=0.8 if jit else 1.0, rng=random.Random(3))
    from packnet_sfm_amd.utils.misc import parse_crop_borders
    box = parse_crop_borders(borders, src)
    H, W = shape if shape else (box[3] - box[1], box[2] - box[0])
    for i in range(n_img):
        slot, b = divmod(i, B)
        d = out["jitter_params"][b] if jit else dict(apply=False)
        o, r = A.train_transform([imgs[i]], box, (H, W), oracle_jitter(d))
        got_o = out["rgb_original"][b] if slot == 0 else out["rgb_context_original"][slot - 1][b]
        got_r = out["rgb"][b] if slot == 0 else out["rgb_context"][slot - 1][b]
        assert got_o.shape == (3, H, W)
        np.testing.assert_array_equal(got_o.cpu().numpy(), o[0], err_msg=f"orig {i}")
        np.testing.assert_array_equal(got_r.cpu().numpy(), r[0], err_msg=f"rgb {i}")
    # intrinsics exactly as the reference's numpy float32 updates (crop :392-410, resize :108-131)
    K = np.array([[721.5, 0, 609.6], [0, 721.5, 172.9], [0, 0, 1]], np.float32)
    if borders:
        K[0, 2] -= box[0]
        K[1, 2] -= box[1]
    if shape:
        sw, sh = W / (box[2] - box[0]), H / (box[3] - box[1])
        K[0, 0] *= sw
        K[1, 1] *= sh
        K[0, 2] *= sw
        K[1, 2] *= sh
    np.testing.assert_array_equal(out["intrinsics"][0].cpu().numpy(), K)
    assert ("intrinsics_full" in out) == bool(borders)


def test_zero_fill_crop_and_determinism(aug):
    """A crop box beyond the image (PIL zero fill), twice: bitwise identical results."""
    g = np.random.default_rng(11)
    imgs = g.integers(0, 256, (4, 37, 61, 3), dtype=np.uint8)
    box = (-9, -4, 70, 45)
    ds = [aug.random_color_jitter_params((0.4, 0.4, 0.4, 0.1, 0.2), 1.0, random.Random(s)) for s in (1, 2)]
    t = torch.from_numpy(imgs).to(DEV)
    o1, r1 = aug.augment_images(t, 2, box, (23, 31), ds)
    o2, r2 = aug.augment_images(t, 2, box, (23, 31), ds)
    assert torch.equal(o1, o2) and torch.equal(r1, r2)
    for i in range(4):
        o, r = A.train_transform([imgs[i]], box, (23, 31), oracle_jitter(ds[i % 2]))
        np.testing.assert_array_equal(o1[i].cpu().numpy(), o[0])
        np.testing.assert_array_equal(r1[i].cpu().numpy(), r[0])


def test_validation_transform(aug):
    g = np.random.default_rng(5)
    imgs = g.integers(0, 256, (2, 375, 1242, 3), dtype=np.uint8)
    out = aug.validation_transforms_batch({"rgb": torch.from_numpy(imgs).to(DEV)}, (192, 640), (-352, 0, 0.5, 1216))
    box = (13, 23, 1229, 375)
    for b in range(2):
        np.testing.assert_array_equal(out["rgb"][b].cpu().numpy(), A.to_tensor(A.resize(A.crop(imgs[b], box), 192, 640)))


def test_rejects_host_tensors(aug):
    with pytest.raises(RuntimeError, match="ROCm"):
        aug.augment_images(torch.zeros(1, 8, 8, 3, dtype=torch.uint8), 1, (0, 0, 8, 8), (4, 4))


def test_per_sample_api_matches_batch(aug):
    """datasets.transforms.train_transforms / get_transforms (per sample, the reference's call
    shape) == one sample of the batched transform with the same random stream."""
    from packnet_sfm_amd.datasets import transforms as T
    g = np.random.default_rng(21)
    frames = [torch.from_numpy(g.integers(0, 256, (375, 1242, 3), dtype=np.uint8)).to(DEV) for _ in range(3)]
    K = torch.tensor([[721.5, 0, 609.6], [0, 721.5, 172.9], [0, 0, 1]])
    sample = {"rgb": frames[0], "rgb_context": frames[1:], "intrinsics": K, "idx": 7}
    tf = T.get_transforms("train", image_shape=(192, 640), jittering=(0.2, 0.2, 0.2, 0.05),
                          crop_train_borders=(-352, 0, 0.5, 1216))
    out = tf(sample, rng=random.Random(9))
    ref = aug.train_transforms_batch({"rgb": frames[0][None], "rgb_context": [f[None] for f in frames[1:]],
                                      "intrinsics": K[None]}, (192, 640), (0.2, 0.2, 0.2, 0.05),
                                     (-352, 0, 0.5, 1216), rng=random.Random(9))
    assert out["idx"] == 7 and out["rgb"].shape == (3, 192, 640) and len(out["rgb_context"]) == 2
    assert torch.equal(out["rgb"], ref["rgb"][0]) and torch.equal(out["rgb_original"], ref["rgb_original"][0])
    for a, b in zip(out["rgb_context"], ref["rgb_context"]):
        assert torch.equal(a, b[0])
    assert torch.equal(out["intrinsics"], ref["intrinsics"][0])
    assert torch.equal(out["intrinsics_full"], K)
    val = T.get_transforms("validation", image_shape=(192, 640), crop_eval_borders=(-352, 0, 0.5, 1216))(
        {"rgb": frames[0], "intrinsics": K})
    assert val["rgb"].shape == (3, 192, 640)
