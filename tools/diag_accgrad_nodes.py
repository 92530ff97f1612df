"""Which parameters' AccumulateGrad nodes survive from one training iteration into the next (the
cause of the stream-mismatch warning when the iterations run on different streams)?  Iteration 0
tags every parameter's AccumulateGrad node (node.metadata); iteration 1's forward reports the
parameters whose node still carries the tag."""
import gc
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
from torch.autograd.graph import get_gradient_edge  # noqa: E402

import __graft_entry__  # noqa: E402
__graft_entry__.build()
import bench  # noqa: E402
from packnet_sfm_amd.trainers import ddp_trainer as T  # noqa: E402

dev = torch.device("cuda:0")


class A:
    depth_net, pose_net, batch, height, width = "ResNetSAN01", "PoseNet", 2, 64, 192


torch.manual_seed(0)
m = bench.to_channels_last(bench.build_model(A, dev))
tr = T.DDPTrainer(m, T.make_optimizer(m, 1e-4, 1e-4, capturable=True), dev, amp_dtype=None, graph=False, flat=True)
b = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)
names = {id(p): n for n, p in m.named_parameters()}
orig = tr._forward_backward
state = {"it": 0}


def fb(batch, progress):
    with torch.autocast("cuda", enabled=False):
        output = tr.ddp(batch, progress=progress)
    for n, p in m.named_parameters():
        if not p.requires_grad:
            continue
        node = get_gradient_edge(p).node
        if state["it"] == 0:
            node.metadata["it0"] = True
        elif node.metadata.get("it0"):
            print(f"[diag] persistent AccumulateGrad: {n}", flush=True)
        del node
    output["loss"].sum().backward()
    return output


tr._forward_backward = fb
tr.train_step(b)
torch.cuda.synchronize()
gc.collect()
state["it"] = 1
tr.train_step(b)
torch.cuda.synchronize()
print("[diag] done", flush=True)
