"""GPU experiment: training-step time of trainer/network variants (graph-captured), one process."""
import json
import sys
import time

sys.path.insert(0, "."); sys.argv = ["bench.py"]
import torch
import torch.nn.functional as F
import bench
import __graft_entry__
__graft_entry__.build()
from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
args = bench.parse()
_orig_bn = torch.nn.BatchNorm2d.forward


def native_bn_forward(self, x):
    with torch.backends.cudnn.flags(enabled=False):
        return _orig_bn(self, x)


res = {}
variants = [("serial", {"overlap": False}), ("overlap", {"overlap": True})]
for name, kw in variants:
    torch.nn.BatchNorm2d.forward = native_bn_forward if kw.get("native_bn") else _orig_bn
    torch.manual_seed(0)
    model = bench.build_model(args, dev).to(memory_format=torch.channels_last)
    model.overlap_pose_net = kw.get("overlap", True)
    batch = bench.synthetic_batch(4, 192, 640, dev, 0, channels_last=True)
    opt = make_optimizer(model, 1e-4, 1e-4, capturable=True, fused=True)
    tr = DDPTrainer(model, opt, dev, amp_dtype=torch.bfloat16, bf16_weights=True)
    try:
        for _ in range(5):
            tr.train_step(batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(40):
            tr.train_step(batch)
        torch.cuda.synchronize()
        res[name] = round(1000 * (time.perf_counter() - t0) / 40, 3)
        res[name + "_loss"] = float(tr.static_output["loss"])
    except Exception as e:
        res[name] = f"ERR {type(e).__name__}: {str(e)[:300]}"
    print(name, res[name], flush=True)
    del tr, model, opt
    torch.cuda.empty_cache()
print(json.dumps(res))
