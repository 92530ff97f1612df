"""GPU experiment: training-step time of network/layout variants (graph-captured), one process."""
import sys, time, json
sys.path.insert(0, "."); sys.argv = ["bench.py"]
import torch
import bench
import __graft_entry__
__graft_entry__.build()
from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = True
args = bench.parse()
res = {}
for name, cl, amp in [("nchw_bf16", False, "bf16"), ("nhwc_bf16", True, "bf16")]:
    torch.manual_seed(0)
    model = bench.build_model(args, dev)
    batch = bench.synthetic_batch(4, 192, 640, dev, 0)
    if cl:
        model = model.to(memory_format=torch.channels_last)
        for k in ("rgb", "rgb_original"):
            batch[k] = batch[k].contiguous(memory_format=torch.channels_last)
        batch["rgb_context"] = [c.contiguous(memory_format=torch.channels_last) for c in batch["rgb_context"]]
        batch["rgb_context_original"] = batch["rgb_context"]
    opt = make_optimizer(model, 1e-4, 1e-4, capturable=True, fused=True)
    tr = DDPTrainer(model, opt, dev, amp_dtype=torch.bfloat16 if amp == "bf16" else None)
    try:
        for _ in range(5):
            tr.train_step(batch)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(30):
            tr.train_step(batch)
        torch.cuda.synchronize()
        res[name] = round(1000 * (time.perf_counter() - t0) / 30, 3)
    except Exception as e:
        res[name] = f"ERR {type(e).__name__}: {str(e)[:200]}"
    print(name, res[name], flush=True)
    del tr, model, opt
    torch.cuda.empty_cache()
print(json.dumps(res))
