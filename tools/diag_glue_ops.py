"""Census of the ATen ops one eager training step dispatches (TorchDispatchMode), with the
Python call site of every fill / zero / copy / cat / elementwise op that is not a convolution or
one of our C-ABI kernels -- to find the glue launches left in the HIP-graph step.

  python tools/diag_glue_ops.py [--depth-net ResNetSAN01] [--batch 4]
Writes gpurun_out/glue_ops.txt.
"""
import argparse
import collections
import os
import sys
import traceback

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
from torch.utils._python_dispatch import TorchDispatchMode  # noqa: E402

import bench  # noqa: E402

SKIP = ("convolution", "cudnn", "miopen", "detach", "view", "_unsafe_view", "t.default", "as_strided",
        "empty", "permute", "expand", "unsqueeze", "squeeze", "slice", "select", "reshape", "alias",
        "transpose", "split", "unbind")


def site():
    fr = [f for f in traceback.extract_stack()[:-3]
          if "packnet-sfm-resnet-san_amd" in f.filename or f.filename.endswith("bench.py")]
    fr = [f for f in fr if "diag_glue_ops" not in f.filename]
    if not fr:
        return "<autograd engine / outside package>"
    return " <- ".join(f"{os.path.basename(f.filename)}:{f.lineno}" for f in reversed(fr[-3:]))


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.ops = collections.Counter()
        self.sites = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        name = str(func)
        self.ops[name] += 1
        if not any(s in name for s in SKIP):
            shp = next((tuple(a.shape) for a in args if isinstance(a, torch.Tensor)), ())
            dt = next((str(a.dtype).replace("torch.", "") for a in args if isinstance(a, torch.Tensor)), "")
            self.sites[(name, site(), f"{dt}{list(shp)}")] += 1
        return func(*args, **(kwargs or {}))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth-net", default="ResNetSAN01")
    ap.add_argument("--pose-net", default="PoseNet")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "glue_ops.txt"))
    a = ap.parse_args()
    ns = argparse.Namespace(depth_net=a.depth_net, pose_net=a.pose_net, batch=a.batch, height=192, width=640,
                            amp="bf16", nchw=False, eager=True)
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = bench.build_model(ns, dev).to(memory_format=torch.channels_last)
    opt = make_optimizer(model, 1e-4, 1e-4, capturable=True, fused=True)
    tr = DDPTrainer(model, opt, dev, amp_dtype=torch.bfloat16, graph=False, flat=True, bf16_weights=True)
    batch = bench.synthetic_batch(a.batch, 192, 640, dev, seed=0, channels_last=True)
    for _ in range(2):
        tr.train_step(batch)
    torch.cuda.synchronize()
    c = Census()
    with c:
        tr.train_step(batch)
    torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    with open(a.out, "w") as f:
        f.write(f"one eager step, {a.depth_net}+{a.pose_net}, B={a.batch}\n=== op counts ===\n")
        for k, v in c.ops.most_common():
            f.write(f"{v:5d}  {k}\n")
        f.write("=== non-view / non-conv ops by call site ===\n")
        for (name, s, shp), v in sorted(c.sites.items(), key=lambda kv: (kv[0][0], -kv[1])):
            f.write(f"{v:4d}  {name:40s} {shp:32s} {s}\n")
    print("wrote", a.out)


if __name__ == "__main__":
    main()
