"""The resident batch gather (include/psfm_augment.h psfm_gather_frames, datasets/synthetic.py
ResidentLoader._gather_hip): one HIP launch per step must write exactly what the index_select +
layout-copy chain writes — every image store in its NCHW and channels_last destinations and the
intrinsics, for single- and multi-camera (DDAD flatten_cameras order) samples.  Bitwise: a gather
is a copy."""
import pytest
import torch

import packnet_sfm_amd  # noqa: F401
from packnet_sfm_amd.datasets.synthetic import ResidentLoader, SyntheticSfmDataset, get_datasampler

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    if not torch.cuda.is_available():
        pytest.skip("needs a ROCm GPU")
    import __graft_entry__
    __graft_entry__.build()
    return torch.device("cuda", 0)


def _dst(B, H, W, dev, split):
    """The trainer's static batch: nets' inputs channels_last beside NCHW loss inputs (split), or one
    NCHW tensor per key (the bench's --nchw layout)."""
    def t(cl):
        x = torch.full((B, 3, H, W), float("nan"), device=dev)
        return x.contiguous(memory_format=torch.channels_last) if cl else x
    d = {"rgb": t(split), "rgb_context": [t(split), t(split)], "intrinsics": torch.full((B, 3, 3), float("nan"), device=dev)}
    d["rgb_original"] = t(False) if split else d["rgb"]
    d["rgb_context_original"] = [t(False) for _ in range(2)] if split else d["rgb_context"]
    return d


@pytest.mark.parametrize("cams,split", [(1, True), (1, False), (4, True)])
def test_hip_gather_equals_index_select(dev, cams, split):
    B, H, W = 2, 24, 40
    ds = SyntheticSfmDataset(8, H, W, 2, cams, seed=3)
    a = ResidentLoader(ds, B, get_datasampler(ds, "train"), dev)
    b = ResidentLoader(ds, B, get_datasampler(ds, "train"), dev)
    b._gather_hip = lambda idx, dst: False          # the index_select chain
    calls = []
    orig = a._gather_hip
    a._gather_hip = lambda idx, dst: calls.append(orig(idx, dst)) or calls[-1]
    for _ in range(5):                               # crosses an epoch boundary (4 steps per epoch)
        da, db = a.next_into(_dst(B * cams, H, W, dev, split)), b.next_into(_dst(B * cams, H, W, dev, split))
        torch.cuda.synchronize()
        for k in ("rgb", "rgb_original", "intrinsics"):
            assert torch.equal(da[k], db[k]), k
            assert da[k].stride() == db[k].stride()
        for k in ("rgb_context", "rgb_context_original"):
            for x, y in zip(da[k], db[k]):
                assert torch.equal(x, y), k
    assert calls and all(c is True for c in calls)   # the HIP gather ran every step
