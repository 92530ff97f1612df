"""Synthetic KITTI / DDAD-shaped training samples, the reference's distributed sampler, and a
HBM-resident loader for the timed training loop.

The reference trains from `OptimizedKITTIDataset` / `DGPDataset` through a `DataLoader` whose
sampler is `DistributedSampler(dataset, shuffle=(mode == 'train'), num_replicas=world_size(),
rank=rank())` (packnet_sfm/models/model_wrapper.py:1138-1144, :1147-1216).  No dataset files
exist here (data readers out of scope), so samples are seeded textures of the
same shapes and keys as `train_transforms` output (datasets/transforms.py:21-50):
'rgb', 'rgb_context', 'rgb_original', 'rgb_context_original', 'intrinsics', 'idx'.

  * `SyntheticSfmDataset(n, H, W)`: sample i is a pure function of (seed, i) — the same on
    every rank, so the sampler's partition (not the seed) decides what a rank trains on;
    `cameras > 1` gives DDAD-style multi-camera samples ([cameras, 3, H, W] per key, per-camera
    intrinsics), which `stack_batch` (models/model_utils.py) folds into the batch dimension
    (packnet_sfm/models/model_utils.py:68-94).
  * `get_datasampler` / `setup_dataloader`: model_wrapper.py:1138-1216 (host DataLoader).
  * `ResidentLoader`: the dataset is materialised on the device once; each step gathers the next
    batch of this rank's sampler partition into caller-owned (e.g. HIP-graph static) tensors
    with `index_select` on device indices — no host sync, no PCIe in the timed loop.
"""
import ctypes

import torch
import torch.nn.functional as F
from torch.utils.data import DataLoader, Dataset
from torch.utils.data.distributed import DistributedSampler

from ..utils.horovod import rank as hvd_rank, world_size as hvd_world_size


def _texture(g, C, H, W):
    base = torch.rand(1, C, max(H // 8, 2), max(W // 8, 2), generator=g)
    img = F.interpolate(base, size=(H, W), mode="bilinear", align_corners=False)[0]
    return (img + 0.05 * torch.randn(C, H, W, generator=g)).clamp(0, 1)


def kitti_intrinsics(H, W):
    """Normalised KITTI pinhole K (fx = 0.58 W, fy = 1.92 H, principal point at the centre)."""
    return torch.tensor([[0.58 * W, 0, 0.5 * W], [0, 1.92 * H, 0.5 * H], [0, 0, 1.0]])


class SyntheticSfmDataset(Dataset):
    def __init__(self, n, height=192, width=640, n_context=2, cameras=1, seed=0):
        self.n, self.H, self.W, self.n_context, self.cameras, self.seed = n, height, width, n_context, cameras, seed

    def __len__(self):
        return self.n

    def __getitem__(self, idx):
        g = torch.Generator().manual_seed(self.seed * 1000003 + idx)
        C, H, W = self.cameras, self.H, self.W

        def frame():
            t = torch.stack([_texture(g, 3, H, W) for _ in range(C)])
            return t if C > 1 else t[0]

        rgb = frame()
        ctx = [frame() for _ in range(self.n_context)]
        K = kitti_intrinsics(H, W)
        if C > 1:  # per-camera principal points (DDAD rigs differ per camera)
            K = K.repeat(C, 1, 1)
            K[:, 0, 2] += torch.linspace(-0.02, 0.02, C) * W
        return {"idx": idx, "rgb": rgb, "rgb_context": ctx, "rgb_original": rgb, "rgb_context_original": ctx,
                "intrinsics": K}


def get_datasampler(dataset, mode):
    """model_wrapper.py:1138-1144."""
    return DistributedSampler(dataset, shuffle=(mode == "train"), num_replicas=hvd_world_size(), rank=hvd_rank())


def setup_dataloader(datasets, batch_size, mode, num_workers=0):
    """model_wrapper.py:1147-1216 (minus the fork's advanced-augmentation collate hooks)."""
    loaders = []
    for ds in datasets:
        sampler = get_datasampler(ds, mode)
        loaders.append(DataLoader(ds, batch_size=batch_size, shuffle=False, pin_memory=False,
                                  num_workers=num_workers, sampler=sampler))
    return loaders


def flatten_cameras(batch):
    """[B, cameras, ...] -> [B * cameras, ...] for every image / intrinsics key (the multi-camera
    batch layout stack_batch produces for B = 1, generalised to any B)."""
    out = dict(batch)
    for k in ("rgb", "rgb_original", "intrinsics"):
        if k in out and out[k].dim() == (5 if k != "intrinsics" else 4):
            out[k] = out[k].flatten(0, 1)
    for k in ("rgb_context", "rgb_context_original"):
        if k in out and out[k][0].dim() == 5:
            out[k] = [c.flatten(0, 1) for c in out[k]]
    return out


class ResidentLoader:
    """Batches of this rank's sampler partition, gathered on the device.

    The whole dataset is materialised on the device once (the sampler reshuffles its global order
    every epoch, so a rank's partition changes between epochs).  `next_into(dst)` writes the next
    batch into the tensors of `dst` (same keys / shapes as a collated batch after
    `flatten_cameras`) with `index_select(..., out=)`: one gather kernel per
    image tensor.  Epochs advance with `sampler.set_epoch` (reshuffle on the host once per epoch,
    indices uploaded asynchronously from pinned memory)."""

    def __init__(self, dataset, batch_size, sampler, device, drop_last=True):
        self.dataset, self.B, self.sampler, self.device = dataset, batch_size, sampler, device
        self.drop_last = drop_last
        samples = [dataset[i] for i in range(len(dataset))]
        cat = lambda ts: torch.stack(ts).to(device)   # noqa: E731
        self.store = {"rgb": cat([s["rgb"] for s in samples]),
                      "rgb_context": [cat([s["rgb_context"][j] for s in samples])
                                      for j in range(len(samples[0]["rgb_context"]))],
                      "intrinsics": cat([s["intrinsics"] for s in samples])}
        self.cameras = getattr(dataset, "cameras", 1)
        self.epoch, self.step_in_epoch, self._idx = 0, 0, None
        self._load_epoch()

    def _load_epoch(self):
        if hasattr(self.sampler, "set_epoch"):
            self.sampler.set_epoch(self.epoch)
        self.partition = list(iter(self.sampler))   # this epoch's sample indices for this rank
        local = torch.tensor(self.partition, dtype=torch.int64)
        n = (len(local) // self.B) * self.B if self.drop_last else len(local)
        self.steps_per_epoch = max(n // self.B, 1)
        self._idx = local[:max(n, self.B)].pin_memory().to(self.device, non_blocking=True) \
            if self.device.type == "cuda" else local[:max(n, self.B)]
        self.step_in_epoch = 0

    def __len__(self):
        return self.steps_per_epoch

    def _sel(self, t, idx, out):
        if self.cameras > 1:   # [n, cams, ...] -> gather samples, flatten cameras into the batch
            src = t.flatten(0, 1)
            cams = torch.arange(self.cameras, device=idx.device)
            idx = (idx[:, None] * self.cameras + cams[None]).reshape(-1)
            t = src
        if out is None:
            return t.index_select(0, idx)
        return torch.index_select(t, 0, idx, out=out) if out.is_contiguous() else out.copy_(t.index_select(0, idx))

    def _gather_hip(self, idx, dst):
        """The whole batch in ONE HIP launch (include/psfm_augment.h psfm_gather_frames): every image
        store into its NCHW (loss) and channels_last (nets) destinations, plus the intrinsics — the
        index_select + layout-copy chain of `_sel` is ~10 launches per step.  False (the chain runs)
        off the GPU or for layouts the kernel does not write."""
        st = self.store
        if self.device.type != "cuda" or "rgb_original" not in dst:
            return False
        keys = [("rgb", "rgb_original", st["rgb"])] + [
            (("rgb_context", j), ("rgb_context_original", j), c) for j, c in enumerate(st["rgb_context"])]

        def get(k):
            return dst[k] if isinstance(k, str) else dst[k[0]][k[1]]

        srcs, nchw, nhwc = [], [], []
        for kn, ko, src in keys:
            a, b = get(kn), get(ko)
            pair = {"nchw": None, "nhwc": None}
            for t in (a, b) if a is not b else (a,):
                if t.dtype != torch.float32 or tuple(t.shape) != (self.B * self.cameras,) + tuple(src.shape[-3:]):
                    return False
                if t.is_contiguous():
                    slot = "nchw"
                elif t.is_contiguous(memory_format=torch.channels_last):
                    slot = "nhwc"
                else:
                    return False
                if pair[slot] is not None:
                    return False
                pair[slot] = t
            srcs.append(src)
            nchw.append(pair["nchw"])
            nhwc.append(pair["nhwc"])
        H, W = srcs[0].shape[-2:]
        if (len(srcs) > 4 or (H * W) % 4 or srcs[0].shape[-3] != 3 or not all(s_.is_contiguous() for s_ in srcs)):
            return False
        # the kernel reads / writes intrinsics as float32 [*, 9] rows indexed by idx * cams + cam
        di, si = dst["intrinsics"], st["intrinsics"]
        n_store = srcs[0].shape[0]
        if (di.dtype != torch.float32 or si.dtype != torch.float32 or not di.is_contiguous() or not si.is_contiguous()
                or tuple(di.shape[-2:]) != (3, 3) or di.numel() != self.B * self.cameras * 9
                or si.numel() != n_store * self.cameras * 9 or di.device != idx.device or si.device != idx.device):
            return False
        from .. import _hip
        P = ctypes.c_void_p * len(srcs)
        _hip.check(_hip.lib().psfm_gather_frames(
            len(srcs), P(*[s_.data_ptr() for s_ in srcs]), P(*[t.data_ptr() if t is not None else None for t in nchw]),
            P(*[t.data_ptr() if t is not None else None for t in nhwc]), _hip.ptr(idx), self.B, self.cameras, H * W,
            _hip.ptr(st["intrinsics"]), _hip.ptr(dst["intrinsics"]), _hip.stream(idx.device)), "psfm_gather_frames")
        return True

    def next_into(self, dst=None):
        if self.step_in_epoch >= self.steps_per_epoch:
            self.epoch += 1
            self._load_epoch()
        i = self.step_in_epoch
        idx = self._idx[i * self.B:(i + 1) * self.B]
        self.step_in_epoch += 1
        st = self.store
        if dst is None:
            rgb = self._sel(st["rgb"], idx, None)
            ctx = [self._sel(c, idx, None) for c in st["rgb_context"]]
            return {"rgb": rgb, "rgb_context": ctx, "rgb_original": rgb, "rgb_context_original": ctx,
                    "intrinsics": self._sel(st["intrinsics"], idx, None)}
        if self._gather_hip(idx, dst):
            return dst
        self._sel(st["rgb"], idx, dst["rgb"])
        for j, c in enumerate(st["rgb_context"]):
            self._sel(c, idx, dst["rgb_context"][j])
        for k, src in (("rgb_original", "rgb"), ("rgb_context_original", "rgb_context")):
            if k in dst and dst[k] is not dst[src]:   # loss inputs (NCHW) beside the nets' layout
                if k == "rgb_original":
                    self._sel(st["rgb"], idx, dst[k])
                else:
                    for j, c in enumerate(st["rgb_context"]):
                        if dst[k][j] is not dst["rgb_context"][j]:
                            self._sel(c, idx, dst[k][j])
        self._sel(st["intrinsics"], idx, dst["intrinsics"])
        return dst
