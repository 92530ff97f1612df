"""Which phase of the graph trainer emits the AccumulateGrad stream-mismatch warning?"""
import os
import sys
import warnings

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import __graft_entry__  # noqa: E402
__graft_entry__.build()
import bench  # noqa: E402
from packnet_sfm_amd.trainers import ddp_trainer as T  # noqa: E402

dev = torch.device("cuda:0")


class A:
    depth_net, pose_net, batch, height, width = "ResNetSAN01", "PoseNet", 2, 64, 192


torch.manual_seed(0)
m = bench.to_channels_last(bench.build_model(A, dev))
tr = T.DDPTrainer(m, T.make_optimizer(m, 1e-4, 1e-4, capturable=True, fused=True), dev, amp_dtype=torch.bfloat16,
                  graph=True, bf16_weights=True)
b = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)
orig_fb = tr._forward_backward
phase = {"name": "?", "i": 0}


def fb(batch, progress):
    phase["i"] += 1
    with warnings.catch_warnings(record=True) as w:
        warnings.simplefilter("always")
        out = orig_fb(batch, progress)
    for x in w:
        if "AccumulateGrad" in str(x.message):
            print(f"[diag] warning in forward_backward call {phase['i']} "
                  f"(capturing={torch.cuda.is_current_stream_capturing()})", flush=True)
    return out


tr._forward_backward = fb
tr.train_step(b)
tr.train_step(b)
torch.cuda.synchronize()
print("[diag] done", phase["i"], "forward_backward calls", flush=True)
