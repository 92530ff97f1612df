"""Which forward op produced the gradient that hits the AccumulateGrad stream-mismatch warning at
capture?  The warning is turned into an error inside backward under anomaly mode, so the error
carries the forward stack trace of the node that was running."""
import os
import sys
import traceback
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
m.overlap_pose_net = os.environ.get("DIAG_OVERLAP", "1") == "1"
tr = T.DDPTrainer(m, T.make_optimizer(m, 1e-4, 1e-4, capturable=True), dev, amp_dtype=None, graph=False, flat=True)
b = bench.synthetic_batch(2, 64, 192, dev, seed=0, channels_last=True)
s = torch.cuda.Stream(device=dev)
for it in range(3):
    # iteration 0 on a side stream (the capture's warm-up), 1 and 2 on another stream
    st = s if it == 0 else torch.cuda.Stream(device=dev)
    st.wait_stream(torch.cuda.current_stream(dev))
    with torch.cuda.stream(st), warnings.catch_warnings():
        warnings.simplefilter("ignore")
        warnings.filterwarnings("error", message=".*AccumulateGrad.*")
        try:
            with torch.autograd.detect_anomaly(check_nan=False):
                tr.train_step(b)
            print(f"[diag] iteration {it}: no warning", flush=True)
        except Exception as e:   # noqa: BLE001
            print(f"[diag] iteration {it}: {type(e).__name__}", flush=True)
            print("".join(traceback.format_exception(e))[-6000:], flush=True)
    torch.cuda.current_stream(dev).wait_stream(st)
    torch.cuda.synchronize()
