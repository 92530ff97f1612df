"""Attribute the eager training step's GPU kernels to PyTorch ops (torch.profiler): which ops
launch the casts / copies / reductions around the MIOpen convolutions.

  python tools/op_profile.py [--depth-net ResNetSAN01] [--steps 3]
Writes gpurun_out/op_profile.txt (top ops by device time, self and total, with call counts).
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import bench  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--depth-net", default="ResNetSAN01")
    ap.add_argument("--pose-net", default="PoseNet")
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "op_profile.txt"))
    a = ap.parse_args()
    ns = argparse.Namespace(depth_net=a.depth_net, pose_net=a.pose_net, batch=a.batch, height=192, width=640,
                            amp="bf16", nchw=False, eager=True)
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    dev = torch.device("cuda", 0)
    from packnet_sfm_amd.networks.layers import fused   # the bench's default net epilogues
    fused.FUSE.update(bias=True, bn=False, gn=True)
    fused.UPCAT = True
    fused.ADD_RELU = True
    torch.manual_seed(0)
    torch.backends.cudnn.benchmark = True
    model = bench.to_channels_last(bench.build_model(ns, dev))
    opt = make_optimizer(model, 1e-4, 1e-4, capturable=True, fused=True)
    tr = DDPTrainer(model, opt, dev, amp_dtype=torch.bfloat16, graph=False, flat=True, bf16_weights=True)
    batch = bench.synthetic_batch(a.batch, 192, 640, dev, seed=0, channels_last=True)
    for _ in range(3):
        tr.train_step(batch)
    torch.cuda.synchronize()
    from torch.profiler import ProfilerActivity, profile
    with profile(activities=[ProfilerActivity.CPU, ProfilerActivity.CUDA], record_shapes=True, with_stack=True) as prof:
        for _ in range(a.steps):
            tr.train_step(batch)
        torch.cuda.synchronize()
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    ka = prof.key_averages()
    with open(a.out, "w") as f:
        f.write(f"{a.steps} eager steps, {a.depth_net}+{a.pose_net}, B={a.batch}\n")
        f.write("=== by self device time ===\n")
        f.write(ka.table(sort_by="self_device_time_total", row_limit=70, max_name_column_width=70))
        f.write("\n=== by total device time ===\n")
        f.write(ka.table(sort_by="device_time_total", row_limit=70, max_name_column_width=70))
        f.write("\n=== by input shape ===\n")
        kg = prof.key_averages(group_by_input_shape=True)
        f.write(kg.table(sort_by="self_device_time_total", row_limit=80, max_name_column_width=40,
                         max_shapes_column_width=90))
        f.write("\n=== by stack (5 frames) ===\n")
        ks = prof.key_averages(group_by_stack_n=6)
        f.write(ks.table(sort_by="self_device_time_total", row_limit=60, max_name_column_width=40))
        # launch attribution of the glue kernels: each device kernel is listed under the innermost
        # op that launched it (FunctionEvent.kernels), with the op's input shapes
        from collections import defaultdict
        att = defaultdict(lambda: [0, 0.0])
        glue = ("SubTensorOp", "fillBuffer", "CastTensor", "copyBuffer", "elementwise", "indexSelect", "clamp",
                "BinaryFunctor", "reduce_kernel", "Cast")
        for e in prof.events():
            for k in getattr(e, "kernels", []) or []:
                if any(g in k.name for g in glue):
                    key = (k.name[:48], e.name, str(e.input_shapes)[:110])
                    att[key][0] += 1
                    att[key][1] += k.duration
        f.write("\n=== glue kernels by launching op (per step) ===\n")
        for (kn, op, shp), (n, us) in sorted(att.items(), key=lambda kv: -kv[1][1]):
            f.write(f"{us / a.steps:9.1f} us {n / a.steps:6.1f}x  {kn:48s}  <- {op}  {shp}\n")
    print("wrote", a.out)


if __name__ == "__main__":
    main()
