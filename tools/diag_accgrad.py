"""Which configuration of the graph trainer emits the AccumulateGrad stream-mismatch warning at
capture?  (a) default, (b) pose net on the current stream, (c) gc.collect() before capture,
(d) no autocast (fp32 nets)."""
import gc
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


def run(tag, overlap=True, collect=False, amp=True):
    torch.manual_seed(0)
    m = bench.to_channels_last(bench.build_model(A, dev))
    m.overlap_pose_net = overlap
    tr = T.DDPTrainer(m, T.make_optimizer(m, 1e-4, 1e-4, capturable=True, fused=amp), dev,
                      amp_dtype=torch.bfloat16 if amp else None, graph=True, bf16_weights=amp)
    b = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)
    orig_fb, hits, n = tr._forward_backward, [], [0]

    def fb(batch, progress):
        n[0] += 1
        if collect and torch.cuda.is_current_stream_capturing():
            pass
        with warnings.catch_warnings(record=True) as w:
            warnings.simplefilter("always")
            out = orig_fb(batch, progress)
        if any("AccumulateGrad" in str(x.message) for x in w):
            hits.append((n[0], torch.cuda.is_current_stream_capturing()))
        return out

    tr._forward_backward = fb
    if collect:
        orig_restore = tr._restore

        def restore(snap):
            orig_restore(snap)
            gc.collect()
        tr._restore = restore
    tr.train_step(b)
    tr.train_step(b)
    torch.cuda.synchronize()
    print(f"[diag] {tag}: warnings at forward_backward calls (call, capturing) {hits}", flush=True)


run("default")
run("pose net on the current stream", overlap=False)
run("gc.collect() after the warm-up", collect=True)
run("fp32 nets, torch Adam", amp=False)
