#!/usr/bin/env python3
"""Self-supervised depth training step throughput (BASELINE.json metric) on MI355X.

Workload (BASELINE.json configs[1]): SelfSupModel = ResNetSAN01('18A') depth net + PoseNet,
KITTI-shaped 192x640 RGB triplets (target + 2 contexts), per-GPU batch 4, 4 full-resolution
scales, automask + min-reprojection, Adam.  Nets under bf16 autocast (MIOpen); the photometric
loss (view synthesis + SSIM/L1 + min + smoothness, fwd+bwd) runs in fp32 on the HIP kernels.

  python bench.py [--gpus N --steps K --warmup W]          (N>1: launched by torch.distributed.run)

Prints ONE JSON line on rank 0 with `roofline` (live HIP-event timing of the photometric kernel
group K1+K2+K3) and `cpu_baseline` (the CPU restatement — same nets on CPU + oracle loss — timed
on this host, rank 0 at N=1 only).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training images/sec (whole node), KITTI 640x192; Abs Rel parity vs ref"
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
LOSS_KW = dict(num_scales=4, ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001, C1=1e-4,
               C2=9e-4, photometric_reduce_op="min", disp_norm=True, clip_loss=0.0, progressive_scaling=0.0,
               padding_mode="zeros", automask_loss=True, min_depth=0.5, max_depth=80.0)
N_CTX, N_SCALES = 2, 4


def algorithmic_bytes_per_image(H, W, N=N_CTX, S=N_SCALES):
    """fwd reads target 12 + contexts 12N + sigmoids 4S B/px; bwd re-reads
    them and writes dL/dsig 4S B/px -> H*W*(2*12*(1+N) + 12*S) (= 120 B/px at N=2, S=4)."""
    return H * W * (2 * 12 * (1 + N) + 12 * S)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--batch", type=int, default=4, help="per-GPU batch (train_resnet_san_kitti_tiny.yaml: 4)")
    ap.add_argument("--height", type=int, default=192)
    ap.add_argument("--width", type=int, default=640)
    ap.add_argument("--depth-net", default="ResNetSAN01", choices=["ResNetSAN01", "PackNet01", "DepthResNet"])
    ap.add_argument("--pose-net", default="PoseNet", choices=["PoseNet", "PoseResNet"])
    ap.add_argument("--amp", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=2)
    ap.add_argument("--no-kernel-timing", action="store_true", help="for rocprofv3 runs")
    ap.add_argument("--eager", action="store_true", help="no HIP-graph capture of the step")
    ap.add_argument("--nchw", action="store_true", help="keep the nets in NCHW (default: channels_last)")
    ap.add_argument("--kernel-iters", type=int, default=20, help="timed photometric fwd+bwd launches")
    ap.add_argument("--no-miopen-find", action="store_true",
                    help="torch.backends.cudnn.benchmark = False (MIOpen heuristics instead of find)")
    ap.add_argument("--data-path", default="resident", choices=["resident", "gpu-augment"],
                    help="gpu-augment: every step first runs the reference's train_transforms on the GPU "
                         "(datasets/augmentations.train_transforms_batch) from raw 375x1242 uint8 KITTI-sized "
                         "frames resident in HBM: LANCZOS resize + colour jitter (0.2,0.2,0.2,0.05) + ToTensor")
    ap.add_argument("--fused-nets", action="store_true",
                    help="run the nets' BN/GN/bias+activation epilogues as fused HIP kernels (psfm_netops)")
    return ap.parse_args()


def synthetic_batch(B, H, W, device, seed, channels_last=False):
    """Seeded KITTI-shaped batch (BASELINE.md plan): smooth textures in [0,1], 2 contexts, K.
    Net inputs (`rgb`, `rgb_context`) optionally channels_last (MIOpen NHWC kernels, no layout
    transposes); the loss inputs (`*_original`) stay NCHW for the HIP kernels."""
    g = torch.Generator().manual_seed(seed)

    def tex():
        base = torch.rand(B, 3, max(H // 8, 2), max(W // 8, 2), generator=g)
        img = torch.nn.functional.interpolate(base, size=(H, W), mode="bilinear", align_corners=False)
        return (img + 0.05 * torch.randn(B, 3, H, W, generator=g)).clamp(0, 1)

    rgb, ctx = tex(), [tex() for _ in range(N_CTX)]
    K = torch.tensor([[0.58 * W, 0, 0.5 * W], [0, 1.92 * H, 0.5 * H], [0, 0, 1.0]]).repeat(B, 1, 1)
    to = lambda t: t.to(device).contiguous()  # noqa: E731
    rgb, ctx, K = to(rgb), [to(c) for c in ctx], to(K)
    batch = dict(rgb=rgb, rgb_context=ctx, rgb_original=rgb, rgb_context_original=ctx, intrinsics=K)
    if channels_last:
        cl = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
        batch["rgb"], batch["rgb_context"] = cl(rgb), [cl(c) for c in ctx]
    return batch


def raw_frames(B, device, seed, h=375, w=1242):
    """Seeded decoded-frame stand-ins (uint8 [B,h,w,3], smooth textures) for --data-path gpu-augment."""
    g = torch.Generator().manual_seed(seed)

    def frame():
        base = torch.rand(B, 3, h // 8, w // 8, generator=g)
        img = torch.nn.functional.interpolate(base, size=(h, w), mode="bilinear", align_corners=False)
        img = (img + 0.05 * torch.randn(B, 3, h, w, generator=g)).clamp(0, 1)
        return (img * 255).round().to(torch.uint8).permute(0, 2, 3, 1).contiguous().to(device)

    K = torch.tensor([[721.5, 0, 609.6], [0, 721.5, 172.9], [0, 0, 1.0]]).repeat(B, 1, 1)
    return {"rgb": frame(), "rgb_context": [frame() for _ in range(N_CTX)], "intrinsics": K.to(device)}


def to_channels_last(model):
    """NHWC for every 4-D parameter (the MIOpen NHWC conv kernels); PackNet01's Conv3d weights
    (5-D) stay as they are (Module.to(memory_format=...) refuses a model that has them)."""
    with torch.no_grad():
        for p in model.parameters():
            if p.dim() == 4:   # explicit NHWC strides (also for 1x1 kernels, as Module.to does)
                p.data = torch.empty_like(p.data, memory_format=torch.channels_last).copy_(p.data)
    return model


def build_model(args, device):
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.models.SelfSupModel import SelfSupModel
    from packnet_sfm_amd.networks import load_depth_net, load_pose_net
    model = SelfSupModel(**LOSS_KW, upsample_depth_maps=True, rotation_mode="euler")
    dkw = {"ResNetSAN01": dict(version="18A", min_depth=0.5, max_depth=80.0),
           "PackNet01": dict(version="1A"), "DepthResNet": dict(version="18pt")}[args.depth_net]
    model.add_depth_net(load_depth_net(args.depth_net, **dkw))
    model.add_pose_net(load_pose_net(args.pose_net, **({"nb_ref_imgs": 2} if args.pose_net == "PoseNet"
                                                        else {"version": "18pt"})))
    return model.to(device).train()


def cpu_baseline(args):
    """The reference's CPU training step restated: the same nets on CPU in fp32 + the oracle loss
    (oracle/photometric_oracle.py, fixture-proven equal to the reference), Adam step."""
    from oracle import photometric_oracle as O
    threads = min(16, os.cpu_count() or 1)
    torch.set_num_threads(threads)
    dev = torch.device("cpu")
    model = build_model(args, dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    batch = synthetic_batch(args.batch, args.height, args.width, dev, seed=1234)
    kw = dict(num_scales_=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001, photometric_reduce_op="min",
              automask_loss=True, clip_loss=0.0, min_depth=0.5, max_depth=80.0)

    def step():
        opt.zero_grad(set_to_none=True)
        inv = model.depth_net(batch["rgb"])["inv_depths"]
        inv = [torch.nn.functional.interpolate(i, size=(args.height, args.width), mode="nearest") for i in inv]
        vec = model.pose_net(batch["rgb"], batch["rgb_context"])
        mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(N_CTX)]
        loss = O.photometric_loss(batch["rgb"], batch["rgb_context"], inv, batch["intrinsics"],
                                  batch["intrinsics"], mats, None, **kw)[0]
        loss.sum().backward()
        opt.step()

    def loss_only():
        sig = [torch.rand(args.batch, 1, args.height, args.width, generator=torch.Generator().manual_seed(i))
               .mul(0.19).add(0.01).requires_grad_(True) for i in range(4)]
        vec = torch.zeros(args.batch, N_CTX, 6)
        vec[:, :, 2] = torch.tensor([-1.0, 1.0])
        vec.requires_grad_(True)
        mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(N_CTX)]
        O.photometric_loss(batch["rgb"], batch["rgb_context"], sig, batch["intrinsics"], batch["intrinsics"],
                           mats, None, **kw)[0].sum().backward()

    step()  # warm-up
    t0 = time.perf_counter()
    for _ in range(args.cpu_steps):
        step()
    dt = (time.perf_counter() - t0) / args.cpu_steps
    loss_only()
    t0 = time.perf_counter()
    for _ in range(3):
        loss_only()
    dl = (time.perf_counter() - t0) / 3
    return {"value": round(args.batch / dt, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"{args.cpu_steps} timed steps (+1 warm-up) of the full SelfSupModel step "
                      f"({args.depth_net}+{args.pose_net}, fp32, B={args.batch}, {args.height}x{args.width}, "
                      f"Adam) with the oracle loss",
            "s_per_step": round(dt, 3), "loss_only_images_per_s": round(args.batch / dl, 3)}


def time_photometric_kernels(args, trainer, batch, HP):
    """Live HIP-event timing of the photometric C-ABI calls on this step's own inputs (the depth /
    pose outputs of the last step): one loss fwd+bwd is run with call recording on, then each
    recorded call is captured into a HIP graph and replayed between two HIP events on the replay
    stream (HP.graph_replay_times_us) -> per-call GPU time without host launch gaps, the same
    per-kernel durations rocprofv3 reports for the graph-replayed training step."""
    out = trainer.static_output if trainer.graphs else trainer.model(batch)
    sigs = [s.detach().float().clone().requires_grad_(True) for s in out["inv_depths"]]
    poses = out["poses"]
    loss_fn = trainer.model._photometric_loss

    def fwd_bwd():
        loss_fn(batch["rgb_original"], batch["rgb_context_original"], sigs, batch["intrinsics"],
                batch["intrinsics"], [type(p)(p.mat.detach()) for p in poses])["loss"].sum().backward()

    for _ in range(2):  # warm
        fwd_bwd()
    torch.cuda.synchronize()
    HP.KERNEL_TIMING["record"] = rec = []
    fwd_bwd()
    HP.KERNEL_TIMING["record"] = None
    torch.cuda.synchronize()
    return HP.graph_replay_times_us(rec, sigs[0].device, reps=10, iters=args.kernel_iters)


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    assert world == args.gpus or (world == 1 and args.gpus == 1), \
        f"--gpus {args.gpus} but WORLD_SIZE={world}: launch N>1 with torch.distributed.run"
    torch.cuda.set_device(local_rank)
    device = torch.device("cuda", local_rank)
    if world > 1:
        dist.init_process_group("nccl", device_id=device)

    import __graft_entry__
    if rank == 0 or world == 1:
        __graft_entry__.build()
    if world > 1:
        dist.barrier()
        __graft_entry__.build()
    from packnet_sfm_amd.losses import _hip_photometric as HP
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer

    from packnet_sfm_amd.networks.layers import fused
    fused.ENABLED = bool(args.fused_nets)
    torch.manual_seed(0)  # identical initial weights on every rank (DDP also broadcasts them)
    torch.backends.cudnn.benchmark = not args.no_miopen_find
    model = build_model(args, device)
    if not args.nchw:
        to_channels_last(model)
    opt = make_optimizer(model, 1e-4, 1e-4, capturable=not args.eager, fused=True)
    trainer = DDPTrainer(model, opt, device, amp_dtype=torch.bfloat16 if args.amp == "bf16" else None,
                         graph=not args.eager, bf16_weights=(args.amp == "bf16" and not args.eager))
    batch = synthetic_batch(args.batch, args.height, args.width, device, seed=rank, channels_last=not args.nchw)
    next_batch = lambda: batch  # noqa: E731
    if args.data_path == "gpu-augment":
        import random as _random
        from packnet_sfm_amd.datasets.augmentations import train_transforms_batch
        raw, rng = raw_frames(args.batch, device, seed=rank), _random.Random(rank)

        def next_batch():
            b = train_transforms_batch(raw, (args.height, args.width), (0.2, 0.2, 0.2, 0.05), (), rng=rng)
            return {k: b[k] for k in ("rgb", "rgb_context", "rgb_original", "rgb_context_original", "intrinsics")}

        batch = next_batch()   # the captured (static) batch, in the nets' layout
        if not args.nchw:
            cl = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
            batch["rgb"], batch["rgb_context"] = cl(batch["rgb"]), [cl(c) for c in batch["rgb_context"]]

    for i in range(args.warmup):   # the first steps include MIOpen find and the HIP-graph capture
        t_w = time.perf_counter()
        trainer.train_step(batch)
        torch.cuda.synchronize()
        if rank == 0:
            print(f"[bench] warmup step {i}: {time.perf_counter() - t_w:.2f} s", file=sys.stderr, flush=True)
    trainer.check_finite()

    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        trainer.train_step(next_batch())
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    trainer.check_finite()
    ktimes = {} if args.no_kernel_timing else time_photometric_kernels(args, trainer, batch, HP)
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)

    if rank == 0:
        images = args.batch * world * args.steps
        value = images / elapsed
        per_step_ms = 1000.0 * elapsed / args.steps
        out = {"metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(per_step_ms, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "bf16" if args.amp == "bf16" else "fp32", "data": "synthetic",
               "config": {"workload": f"SelfSupModel {args.depth_net}('18A' if ResNetSAN01) + {args.pose_net}, "
                                      f"KITTI {args.width}x{args.height}, 2 contexts, 4 full-res scales, automask "
                                      f"min-reprojection, Adam (train_resnet_san_kitti_tiny.yaml shapes)",
                          "model": f"{args.depth_net}+{args.pose_net}", "global_batch": args.batch * world,
                          "per_gpu_batch": args.batch, "image_hw": [args.height, args.width],
                          "parallelism": f"dp{world}",
                          "data_path": "resident synthetic batch" if args.data_path == "resident" else
                          "gpu-augment: raw 375x1242 uint8 frames -> train_transforms on the GPU inside every timed step", "net_dtype": args.amp, "loss_dtype": "fp32",
                          "net_layout": "NCHW" if args.nchw else "channels_last",
                          "step": "eager" if args.eager else "hip_graph",
                          "weights_dtype": "bf16 model + fp32 master" if (args.amp == "bf16" and not args.eager)
                          else "fp32",
                          "net_epilogues": "fused HIP (psfm_netops)" if args.fused_nets else "reference op chain",
                          "weights": "random init (no network / checkpoints)"}}
        if ktimes:
            # the photometric fwd+bwd group of one training step (all its HIP launches); the
            # dominant kernel is K12
            group = [k for k in ktimes if k not in ("clip_stats",)]
            group_us = sum(ktimes[k] for k in group)
            bytes_step = algorithmic_bytes_per_image(args.height, args.width) * args.batch
            achieved = bytes_step / (group_us * 1e-6) / 1e9
            dom = "K12_photometric_fwd_grad" if "K12_photometric_fwd_grad" in ktimes else "K2_photometric_bwd"
            traffic = None
            pmc = os.path.join(ROOT, "profiles", "pmc_traffic.json")
            if os.path.exists(pmc):
                with open(pmc) as f:
                    traffic = json.load(f).get("bytes_per_step")
            out["roofline"] = {"bound": "hbm",
                               "kernel": "photometric fwd+bwd group: prepass (K0 automask + sigmoid sums) + K12 "
                                         "fused fwd/bwd sweep + finalize + grad finish + pose reduce",
                               "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                               "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                               "algorithmic_bytes_per_step": bytes_step,
                               "group_us_per_step": round(group_us, 2),
                               "dominant_kernel": dom, "dominant_us_per_step": round(ktimes[dom], 2),
                               "kernels_us_per_step": {k: round(v, 2) for k, v in ktimes.items()},
                               "timing": "HIP events around graph replays of each recorded C-ABI call"}
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
