#!/usr/bin/env python3
"""Self-supervised depth training step throughput (BASELINE.json metric) on MI355X.

Default workload (BASELINE.json configs[1], train_resnet_san_kitti_tiny.yaml shapes):
SelfSupModel = ResNetSAN01('18A') depth net + PoseNet, KITTI-shaped 192x640 RGB triplets
(target + 2 contexts), per-GPU batch 4, 4 full-resolution scales, automask + min-reprojection,
Adam.  Nets under bf16 autocast (MIOpen); the photometric loss (view synthesis + SSIM/L1 + min
+ smoothness, fwd+bwd) in fp32 on the HIP kernels.  Other BASELINE configs: --config.

  python bench.py [--gpus N --steps K --warmup W] [--config NAME]

--gpus N > 1 without a torch.distributed.run environment re-launches itself under
`python -m torch.distributed.run --nproc-per-node N` (before anything touches the GPU) and exits
with its status.  Every rank trains on its DistributedSampler partition of a synthetic dataset
resident in HBM (datasets/synthetic.py); gradients are averaged by one RCCL all-reduce per step.

Prints ONE JSON line on rank 0 with `roofline` (live HIP-event timing of the photometric kernels
on this step's own inputs; the dominant kernel K12 against SURVEY §8(d)'s algorithmic bytes)
and `cpu_baseline` (the CPU restatement — same nets on CPU in fp32 + the oracle loss — timed on
this host's cores, rank 0 at N=1 only).
"""
import argparse
import datetime
import json
import os
import socket
import statistics
import subprocess
import tempfile
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "training images/sec (whole node), KITTI 640x192; Abs Rel parity vs ref"
HBM_PEAK_GBS = 8000.0        # MI355X HBM3E spec peak (MI355X_MICROARCH.md)
SIMDS, CLOCK_HZ = 1024, 2.4e9  # 256 CUs x 4 SIMDs; max shader clock (VALU floor is then a lower bound)
N_CTX, N_SCALES = 2, 4

# BASELINE.json configs -> bench presets (reference YAML in parentheses)
CONFIGS = {
    "overfit": dict(depth_net="DepthResNet", pose_net="PoseResNet", batch=6, height=192, width=640, cameras=1,
                    amp="fp32", min_depth=0.0, max_depth=80.0,
                    yaml="configs/overfit_kitti.yaml (DepthResNet 18pt + PoseResNet 18pt, fp32)"),
    "kitti-resnet-san": dict(depth_net="ResNetSAN01", pose_net="PoseNet", batch=4, height=192, width=640,
                             cameras=1, amp="bf16", min_depth=0.5, max_depth=80.0,
                             yaml="configs/train_resnet_san_kitti_tiny.yaml (ResNetSAN01 18A + PoseNet)"),
    "kitti-packnet": dict(depth_net="PackNet01", pose_net="PoseNet", batch=6, height=192, width=640, cameras=1,
                          amp="bf16", min_depth=0.5, max_depth=80.0,
                          yaml="PackNet01 1A + PoseNet at train_packnet_san_kitti.yaml shapes"),
    "kitti-packnet-san": dict(depth_net="PackNetSAN01", pose_net="PoseNet", batch=6, height=192, width=640,
                              cameras=1, amp="bf16", min_depth=0.5, max_depth=80.0,
                              yaml="configs/train_packnet_san_kitti.yaml (PackNetSAN01 1A RGB path + PoseNet)"),
    "ddad-packnet-san": dict(depth_net="PackNetSAN01", pose_net="PoseNet", batch=1, height=384, width=640,
                             cameras=4, amp="bf16", min_depth=0.5, max_depth=200.0,
                             yaml="configs/train_packnet_san_ddad.yaml (PackNetSAN01 1A, 384x640, "
                                  "cameras 01/05/06/09 per sample)"),
}
DEFAULT_CONFIG = "kitti-resnet-san"


def loss_kw(min_depth, max_depth):
    return dict(num_scales=4, ssim_loss_weight=0.85, occ_reg_weight=0.1, smooth_loss_weight=0.001, C1=1e-4,
                C2=9e-4, photometric_reduce_op="min", disp_norm=True, clip_loss=0.0, progressive_scaling=0.0,
                padding_mode="zeros", automask_loss=True, min_depth=min_depth, max_depth=max_depth)


def algorithmic_bytes_per_image(H, W, N=N_CTX, S=N_SCALES):
    """fwd reads target 12 + contexts 12N + sigmoids 4S B/px; bwd re-reads
    them and writes dL/dsig 4S B/px -> H*W*(2*12*(1+N) + 12*S) (= 120 B/px at N=2, S=4)."""
    return H * W * (2 * 12 * (1 + N) + 12 * S)


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", default=DEFAULT_CONFIG, choices=sorted(CONFIGS))
    ap.add_argument("--batch", type=int, default=None, help="per-GPU samples (preset: the config's YAML)")
    ap.add_argument("--cameras", type=int, default=None, help="cameras per sample (DDAD: 4)")
    ap.add_argument("--height", type=int, default=None)
    ap.add_argument("--width", type=int, default=None)
    ap.add_argument("--depth-net", default=None, choices=["ResNetSAN01", "PackNet01", "PackNetSAN01", "DepthResNet"])
    ap.add_argument("--pose-net", default=None, choices=["PoseNet", "PoseResNet"])
    ap.add_argument("--amp", default=None, choices=["bf16", "fp32"])
    ap.add_argument("--dist-backend", default="nccl", choices=["nccl", "gloo"],
                    help="gloo: rehearse N>1 on one GPU (ranks share the device, host all-reduce)")
    ap.add_argument("--comm", default="auto", choices=["auto", "split", "graph", "overlap"],
                    help="split: all_reduce between two graph replays (no collective inside a graph); "
                         "graph: captured into the step graph after the backward; overlap: bucketed, "
                         "launched from gradient hooks during the backward on a side stream inside the "
                         "step graph; auto (default): at N > 1 over RCCL every rank first runs one "
                         "short-lived child that checks the overlap path on this node "
                         "(trainers/comm_probe.py) — overlap if all pass, split otherwise (config.comm "
                         "says which and why); N = 1 has no collective")
    ap.add_argument("--comm-probe", action="store_true", help=argparse.SUPPRESS)   # the probe child
    ap.add_argument("--comm-probe-timeout", type=float, default=240.0,
                    help="seconds before a hung probe child is killed (-> split)")
    ap.add_argument("--probe-only", action="store_true",
                    help="run the --comm auto selection, print it as JSON on rank 0, exit (no training)")
    ap.add_argument("--probe-report", default=None, help=argparse.SUPPRESS)   # probe child: rank 0's info as JSON
    ap.add_argument("--probe-backend", default=None, choices=["nccl", "gloo"],
                    help="backend of the probe children (default: --dist-backend; gloo = CPU, tests)")
    ap.add_argument("--force-comm", action="store_true",
                    help="run the all-reduce path at N=1 too (world-size-1 RCCL group): its cost on one GPU")
    ap.add_argument("--bucket-mb", type=float, default=16.0, help="comm=overlap bucket size")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-steps", type=int, default=5, help="timed CPU steps (median; +1 warm-up)")
    ap.add_argument("--no-kernel-timing", action="store_true", help="for rocprofv3 runs")
    ap.add_argument("--eager", action="store_true", help="no HIP-graph capture of the step")
    ap.add_argument("--nchw", action="store_true", help="keep the nets in NCHW (default: channels_last)")
    ap.add_argument("--kernel-iters", type=int, default=20, help="timed photometric fwd+bwd launches")
    ap.add_argument("--no-miopen-find", action="store_true",
                    help="torch.backends.cudnn.benchmark = False (MIOpen heuristics instead of find)")
    ap.add_argument("--deterministic", default="none", choices=["none", "cudnn", "all"],
                    help="cudnn: torch.backends.cudnn.deterministic = True, as the reference trainer sets "
                         "(horovod_trainer.py:23); all: torch.use_deterministic_algorithms(True).  Both "
                         "restrict MIOpen to its deterministic solvers: 4.4 -> 1011 ms/step on MI355X "
                         "(profiles/r02_determinism.json), so the bench uses MIOpen's fast solvers")
    ap.add_argument("--data-path", default="sampler", choices=["sampler", "resident", "gpu-augment"],
                    help="sampler: every step gathers the next batch of this rank's DistributedSampler "
                         "partition of a synthetic dataset resident in HBM; resident: one fixed batch; "
                         "gpu-augment: the reference's train_transforms on the GPU from raw 375x1242 uint8 "
                         "frames inside every timed step")
    ap.add_argument("--fused-nets", default="bias,gn,bn",
                    help="net epilogues as fused HIP kernels (psfm_netops): none | all | a comma list of "
                         "bias (conv bias + ReLU/sigmoid), bn (BatchNorm + ReLU [+ identity]: the one-launch "
                         "resident kernels where they hold the layer, MIOpen's BatchNorm elsewhere), bnall (every "
                         "shape the library's fused BatchNorm takes: A/B builds add the two-launch form), "
                         "gn (GroupNorm + ReLU); default: the measured winners (networks/layers/fused.py FUSE)")
    ap.add_argument("--no-add-relu", action="store_true",
                    help="BasicBlock tail relu(bn2 + identity) as the torch op chain instead of psfm_add_relu")
    ap.add_argument("--pose-first", action="store_true",
                    help="enqueue the pose net's branch before the depth net (A/B of the step graph's node order)")
    ap.add_argument("--no-net-inputs", action="store_true",
                    help="the nets' input normalisation / concatenation + autocast casts as ATen ops instead of "
                         "psfm_normalize_bf16 / psfm_cat_channels_bf16")
    ap.add_argument("--no-stem-pool", action="store_true",
                    help="stem relu + max-pool as psfm_add_relu + ATen's max-pool instead of psfm_relu_maxpool")
    ap.add_argument("--no-fork", action="store_true",
                    help="tensors with several consumers as the plain op output (autograd sums their gradients "
                         "with add kernels) instead of forked views summed by the producer's backward kernel")
    ap.add_argument("--no-hip-gather", action="store_true",
                    help="resident batch gather as index_select + layout copies instead of psfm_gather_frames")
    ap.add_argument("--no-upcat", action="store_true",
                    help="DepthDecoder upsample + cat as the torch op chain instead of psfm_upcat")
    args = ap.parse_args(argv)
    preset = CONFIGS[args.config]
    for k in ("batch", "cameras", "height", "width", "depth_net", "pose_net", "amp"):
        if getattr(args, k) is None:
            setattr(args, k, preset[k])
    args.min_depth, args.max_depth, args.yaml = preset["min_depth"], preset["max_depth"], preset["yaml"]
    return args


def source_hash():
    """sha256 (16 hex) of the HIP library's sources — the hash build() compiles into the library
    (psfm_version()) and the code revision a stamped profile was taken on."""
    import __graft_entry__
    return __graft_entry__.source_hash()


def config_key(args):
    """Identifies the workload of a stamped profile file (profiles/pmc/<key>.json)."""
    return (f"{args.depth_net}+{args.pose_net}_B{args.batch}x{args.cameras}_{args.height}x{args.width}_{args.amp}"
            f"{'_nchw' if args.nchw else ''}")


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def relaunch_distributed(args):
    """`bench.py --gpus N` outside torch.distributed.run: start one process per GPU as a CHILD
    (nothing here has touched the GPU) and return its exit status."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.call(cmd, env=env)


def launch_comm_probe(args, rank, world, local_rank, port, backend, report=None):
    """Start THIS rank's probe child (bench.py --comm-probe: trainers/comm_probe.py) in its own
    session and return its exit status (124 after a kill at --comm-probe-timeout).  The children
    form their own process group on `port`; nothing of theirs lives on in this process."""
    import signal
    env = {k: v for k, v in os.environ.items() if not k.startswith("TORCHELASTIC")}
    env.update(RANK=str(rank), WORLD_SIZE=str(world), LOCAL_RANK=str(local_rank), MASTER_ADDR="127.0.0.1",
               MASTER_PORT=str(port), HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    # the child re-parses this run's own arguments (config, batch, --bucket-mb: the probe cuts the
    # same buckets) with the probe flags last
    cmd = [sys.executable, os.path.abspath(__file__), *sys.argv[1:], "--comm-probe", "--gpus", str(world),
           "--dist-backend", backend] + (["--probe-report", report] if report else [])
    p = subprocess.Popen(cmd, env=env, start_new_session=True, stdout=sys.stderr, stderr=sys.stderr)
    try:
        return p.wait(timeout=args.comm_probe_timeout)
    except subprocess.TimeoutExpired:
        os.killpg(p.pid, signal.SIGKILL)
        p.wait()
        return 124


def choose_comm(store, rank, world, run_child):
    """--comm auto at N > 1: rank 0 publishes a free port for the probe children's own process
    group, every rank runs its child (run_child(port) -> exit status) and publishes the status, and
    every rank reads all of them — so all ranks pick the same path: 'overlap' when every child
    passed, else 'split'.  Returns (comm, note for config.comm)."""
    if rank == 0:
        store.set("psfm_probe_port", str(_free_port()))
    port = int(store.get("psfm_probe_port"))
    rc = run_child(port)
    store.set(f"psfm_probe_rc_{rank}", str(int(rc)))
    rcs = [int(store.get(f"psfm_probe_rc_{r}")) for r in range(world)]
    bad = {r: c for r, c in enumerate(rcs) if c != 0}
    if not bad:
        return "overlap", f"auto: overlap probe passed on {world} ranks"
    return "split", f"auto: overlap probe failed (rank: exit status {bad}), split"


def param_shapes(args):
    """(depth-net, pose-net) shapes, in order, of this run's parameters that receive a gradient in its
    step (the trainer buckets only those; ResNetSAN01's sparse-branch blend weights get none on the
    RGB path): the model built and run forward + backward on the meta device (no memory, no kernels).
    The probe's ShapeNet stands in for the model with them."""
    with torch.device("meta"):
        m = build_model(args, torch.device("meta"))
        x = torch.empty(1, 3, args.height, args.width)
        inv = m.depth_net(x)["inv_depths"]
        vec = m.pose_net(x, [x] * N_CTX)
        (sum(i.float().mean() for i in inv) + vec.float().mean()).backward()
    used = lambda net: [tuple(p.shape) for p in net.parameters() if p.grad is not None]  # noqa: E731
    return used(m.depth_net), used(m.pose_net)


def comm_probe_main(args, world, rank, local_rank):
    """The probe child: its own process group, trainers/comm_probe.run_probe, exit status."""
    if os.environ.get("PSFM_TEST_PROBE_FAIL_RANK") == str(rank):   # tests/test_distributed.py: a failing child
        print(f"[comm probe] rank {rank}: failing on request (test)", file=sys.stderr, flush=True)
        return 3
    backend = args.dist_backend
    if backend == "nccl":
        device = torch.device("cuda", local_rank % torch.cuda.device_count())
        torch.cuda.set_device(device)
        dist.init_process_group("nccl", device_id=device)
    else:
        device = torch.device("cpu")
        dist.init_process_group("gloo")
    rc = 0
    try:
        import __graft_entry__
        __graft_entry__.build()   # a no-op: the training ranks built before starting the probe
        from packnet_sfm_amd.trainers.comm_probe import run_probe
        info = run_probe(device, bucket_mb=args.bucket_mb, shapes=param_shapes(args))
        if rank == 0 and args.probe_report:
            with open(args.probe_report, "w") as f:
                json.dump(info, f)
        info.pop("cuts")
        print(f"[comm probe] rank {rank}: {json.dumps(info)}", file=sys.stderr, flush=True)
    except Exception as e:  # noqa: BLE001  (any failure means: do not use the overlap path)
        print(f"[comm probe] rank {rank}: FAILED {type(e).__name__}: {e}", file=sys.stderr, flush=True)
        rc = 1
    finally:
        dist.destroy_process_group()
    return rc


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
        net_layout(batch)
    return batch


def net_layout(batch):
    """The nets' inputs in channels_last beside the NCHW loss inputs (separate tensors)."""
    cl = lambda t: t.contiguous(memory_format=torch.channels_last)  # noqa: E731
    if batch["rgb"] is batch.get("rgb_original"):
        batch["rgb"] = torch.empty_like(batch["rgb"], memory_format=torch.channels_last).copy_(batch["rgb"])
    else:
        batch["rgb"] = cl(batch["rgb"])
    batch["rgb_context"] = [torch.empty_like(c, memory_format=torch.channels_last).copy_(c)
                            for c in batch["rgb_context"]]
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
    """NHWC for every 4-D parameter (the MIOpen NHWC conv kernels); Conv3d weights (5-D) stay as
    they are (Module.to(memory_format=...) refuses a model that has them)."""
    with torch.no_grad():
        for p in model.parameters():
            if p.dim() == 4:   # explicit NHWC strides (also for 1x1 kernels, as Module.to does)
                p.data = torch.empty_like(p.data, memory_format=torch.channels_last).copy_(p.data)
    return model


def build_model(args, device):
    import packnet_sfm_amd  # noqa: F401
    from packnet_sfm_amd.models.SelfSupModel import SelfSupModel
    from packnet_sfm_amd.networks import load_depth_net, load_pose_net
    mn, mx = getattr(args, "min_depth", 0.5), getattr(args, "max_depth", 80.0)
    model = SelfSupModel(**loss_kw(mn, mx), upsample_depth_maps=True, rotation_mode="euler")
    dkw = {"ResNetSAN01": dict(version="18A", min_depth=mn, max_depth=mx),
           "PackNet01": dict(version="1A"), "PackNetSAN01": dict(version="1A", dropout=0.5),
           "DepthResNet": dict(version="18pt")}[args.depth_net]
    model.add_depth_net(load_depth_net(args.depth_net, **dkw))
    model.add_pose_net(load_pose_net(args.pose_net, **({"nb_ref_imgs": 2} if args.pose_net == "PoseNet"
                                                        else {"version": "18pt"})))
    return model.to(device).train()


def host_cores():
    """Cores this job may use on the host: the affinity mask, capped by a cgroup CPU quota and by
    the box's per-GPU share (OMP_NUM_THREADS, set by the GPU pool)."""
    n = len(os.sched_getaffinity(0))
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            n = min(n, max(1, int(q) // int(p)))
    except (OSError, ValueError):
        pass
    omp = os.environ.get("OMP_NUM_THREADS")
    if omp and omp.isdigit() and int(omp) > 0:
        n = min(n, int(omp))
    return max(1, n)


def cpu_baseline(args):
    """The reference's CPU training step restated: the same nets on CPU in fp32 + the oracle loss
    (oracle/photometric_oracle.py, fixture-proven equal to the reference), Adam step.  1 warm-up
    + `cpu_steps` timed steps, median."""
    from oracle import photometric_oracle as O
    threads = host_cores()
    torch.set_num_threads(threads)
    dev = torch.device("cpu")
    model = build_model(args, dev)
    opt = torch.optim.Adam(model.parameters(), lr=1e-4)
    B = args.batch * args.cameras
    batch = synthetic_batch(B, args.height, args.width, dev, seed=1234)
    kw = dict(num_scales_=4, ssim_loss_weight=0.85, smooth_loss_weight=0.001, photometric_reduce_op="min",
              automask_loss=True, clip_loss=0.0, min_depth=args.min_depth, max_depth=args.max_depth)

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
        g = torch.Generator().manual_seed(5)
        sig = [torch.rand(B, 1, args.height, args.width, generator=g).mul(0.19).add(0.01).requires_grad_(True)
               for _ in range(4)]
        vec = torch.zeros(B, N_CTX, 6)
        vec[:, :, 2] = torch.tensor([-1.0, 1.0])
        vec.requires_grad_(True)
        mats = [O.pose_vec_to_mat(vec[:, j]) for j in range(N_CTX)]
        O.photometric_loss(batch["rgb"], batch["rgb_context"], sig, batch["intrinsics"], batch["intrinsics"],
                           mats, None, **kw)[0].sum().backward()

    def timed(fn, n):
        fn()  # warm-up
        ts = []
        for _ in range(n):
            t0 = time.perf_counter()
            fn()
            ts.append(time.perf_counter() - t0)
        return statistics.median(ts)

    dt = timed(step, args.cpu_steps)
    dl = timed(loss_only, args.cpu_steps)
    return {"value": round(B / dt, 4), "unit": "images/s", "cores": threads, "kind": "port",
            "sample": f"median of {args.cpu_steps} timed steps (+1 warm-up) of the full SelfSupModel training "
                      f"step ({args.depth_net}+{args.pose_net}, fp32, {B} images of {args.height}x{args.width}, "
                      f"Adam) with the oracle loss, {threads} threads",
            "s_per_step": round(dt, 3), "loss_only_images_per_s": round(B / dl, 3),
            "cores_note": "host_cores(): affinity mask, capped by the cgroup quota and the box's per-GPU share "
                          "(OMP_NUM_THREADS)"}


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


def k12_in_step(trainer, next_batch, device, reps=10):
    """K12's duration INSIDE the training step: `reps` more step replays (after the timed region)
    with the library's per-wave stamps on (psfm_k12_stamps: each K12 wave writes the constant
    100 MHz clock at its start and end); the launch span = last end - first start.  This is the
    kernel as it runs in the step graph — beside the pose branch, after the depth net — not an
    isolated replay of it."""
    from packnet_sfm_amd import _hip
    L = _hip.lib()
    cap = 1 << 16
    buf = torch.zeros(cap, 2, dtype=torch.int64, device=device)
    st = _hip.stream(device)
    _hip.check(L.psfm_k12_stamps(_hip.ptr(buf), cap, st), "psfm_k12_stamps")
    spans, wave_mean, wave_max, nwaves = [], [], [], 0
    try:
        for _ in range(reps):
            buf.zero_()
            trainer.train_step(next_batch())
            torch.cuda.synchronize()
            b = buf.cpu()
            used = b[:, 0] > 0
            if not bool(used.any()):   # this step does not run the K12 path
                return None
            s0, e1 = b[used, 0], b[used, 1]
            spans.append(float(e1.max() - s0.min()) * 0.01)   # 100 MHz ticks -> us
            d = (e1 - s0).double() * 0.01
            wave_mean.append(float(d.mean()))
            wave_max.append(float(d.max()))
            nwaves = int(used.sum())
        if os.environ.get("PSFM_STAMP_DUMP"):   # the last step's per-wave stamps, for tools/k12_stamps.py
            import numpy as np
            np.save(os.environ["PSFM_STAMP_DUMP"], b[: int(used.nonzero().max()) + 1].numpy())
    finally:
        _hip.check(L.psfm_k12_stamps(None, 0, st), "psfm_k12_stamps")
    return {"us_mean": round(statistics.mean(spans), 2), "us_median": round(statistics.median(spans), 2),
            "us_min": round(min(spans), 2), "us_max": round(max(spans), 2), "reps": reps, "waves": nwaves,
            "wave_us_mean": round(statistics.mean(wave_mean), 2), "wave_us_max": round(max(wave_max), 2),
            "timing": "per-wave s_memrealtime stamps (100 MHz) of K12 inside the replayed step graph: "
                      "last wave end - first wave start, mean over reps extra steps after the timed region"}


def stamped_profile(args):
    """profiles/pmc/<config_key>.json written by tools/pmc_bench.py from rocprofv3 --pmc passes over
    THIS command's workload on THIS source revision; (None, path, why) when no file carries this
    config's key or its source hash differs from the library built from the current sources."""
    path = os.path.join(ROOT, "profiles", "pmc", config_key(args) + ".json")
    if not os.path.exists(path):
        return None, path, "absent for this config"
    with open(path) as f:
        prof = json.load(f)
    if prof.get("config_key") != config_key(args):
        return None, path, "config key mismatch"
    if prof.get("source_hash") != source_hash():
        return None, path, f"stale: taken on sources {prof.get('source_hash')}, library built from {source_hash()}"
    return prof, path, None


def rocprof_k12(args):
    """K12's mean dispatch-to-completion duration inside the step, from the rocprofv3 kernel-trace
    step summary of THIS config on THIS source revision (profiles/rocprof/<config_key>.json, written
    by tools/rocprof_stamp.py from a tools/r5_bench.sh --prof run); None when absent or stale."""
    path = os.path.join(ROOT, "profiles", "rocprof", config_key(args) + ".json")
    if not os.path.exists(path):
        return None, path
    with open(path) as f:
        prof = json.load(f)
    if prof.get("config_key") != config_key(args) or prof.get("source_hash") != source_hash():
        return None, path
    return prof, path


def roofline(args, ktimes, instep=None):
    """Dominant kernel K12 (the fused warp + SSIM + min + smoothness fwd/bwd sweep) against
    SURVEY §8(d)'s algorithmic bytes of the photometric fwd+bwd per image, timed IN the step
    (k12_in_step) when available, the isolated graph replay beside it; the whole photometric
    group beside it; HBM traffic and VALU occupancy from the stamped PMC profile of this config."""
    images = args.batch * args.cameras
    bytes_step = algorithmic_bytes_per_image(args.height, args.width) * images
    group_us = sum(v for k, v in ktimes.items() if k != "clip_stats")
    dom = "K12_photometric_fwd_grad" if "K12_photometric_fwd_grad" in ktimes else "K2_photometric_bwd"
    iso_us = ktimes[dom]
    # the LARGEST of the available K12 durations: the in-step wave-stamp span
    # (first wave start -> last wave end), the isolated graph replay (HIP events), and rocprof's
    # in-step dispatch-to-completion figure of the stamped kernel trace for this config / sources
    cands = {"isolated graph replay (HIP events)": iso_us}
    if instep and dom == "K12_photometric_fwd_grad":
        cands["in step (per-wave clock stamps inside the step graph)"] = instep["us_mean"]
    rp, rp_path = rocprof_k12(args)
    if rp and dom == "K12_photometric_fwd_grad":
        cands["in step, rocprofv3 kernel trace (dispatch to completion, %s)" % os.path.relpath(rp_path, ROOT)] = \
            rp["k12_us_mean"]
    dom_timing, dom_us = max(cands.items(), key=lambda kv: kv[1])
    achieved = bytes_step / (dom_us * 1e-6) / 1e9
    out = {"bound": "hbm", "kernel": dom, "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": None,
           "algorithmic_bytes_per_launch": bytes_step,
           "algorithmic_bytes_note": "SURVEY §8(d): H*W*(2*12*(1+N) + 12*S) B per image (120 B/px), x images "
                                     "per launch",
           "dominant_us_per_launch": round(dom_us, 2),
           "dominant_timing": dom_timing + " — the largest of " + ", ".join(
               f"{k.split(' (')[0]} {v:.2f}" for k, v in cands.items()),
           "isolated_us_per_launch": round(iso_us, 2),
           "in_step": instep,
           "group": {"kernels": "prepass (K0 automask + sigmoid sums) + K12 + finalize + grad finish + pose reduce",
                     "us_per_step": round(group_us, 2),
                     "achieved": round(bytes_step / (group_us * 1e-6) / 1e9, 1),
                     "frac": round(bytes_step / (group_us * 1e-6) / 1e9 / HBM_PEAK_GBS, 4)},
           "kernels_us_per_step": {k: round(v, 2) for k, v in ktimes.items()},
           "timing": "kernels_us_per_step / group / isolated_us_per_launch: HIP events around graph replays "
                     "of each recorded C-ABI call (replay stream)"}
    prof, path, why = stamped_profile(args)
    out["profile"] = os.path.relpath(path, ROOT) + ("" if prof else f" ({why}: traffic null)")
    out["source_hash"] = source_hash()
    if prof:
        k = prof["kernels"].get(dom)
        if k and k.get("hbm_bytes") is not None:
            out["traffic"] = int(k["hbm_bytes"])
            out["traffic_vs_algorithmic"] = round(k["hbm_bytes"] / bytes_step, 3)
        if k and k.get("SQ_ACTIVE_INST_VALU") is not None:
            insts = k.get("SQ_INSTS_VALU") or k["SQ_ACTIVE_INST_VALU"]
            # a wave64 VALU instruction holds a SIMD for 2 cycles when two waves interleave, and a lone
            # wave issues one every 4 cycles (MI355X_MICROARCH.md, wave scheduling)
            t2 = insts * 2 / SIMDS / CLOCK_HZ * 1e6
            t4 = insts * 4 / SIMDS / CLOCK_HZ * 1e6
            v = {"insts": insts, "active_quad_cycles": k["SQ_ACTIVE_INST_VALU"],
                 "simd_floor_us_2cyc": round(t2, 2), "lone_wave_floor_us_4cyc": round(t4, 2),
                 "note": "VALU instructions x 2 (or 4) cycles / 1024 SIMDs / 2.4 GHz: the launch's VALU issue time "
                         "at perfect 2-wave interleave (or one wave per SIMD); compare dominant_us_per_launch"}
            # the kernel's distance from its own VALU issue floor (2-wave interleave): 1.0 = VALU-issue bound
            v["valu_floor_us_over_dominant_us"] = round(t2 / dom_us, 3)
            if k.get("SQ_WAVE_CYCLES"):
                v["wave_valu_frac"] = round(k["SQ_ACTIVE_INST_VALU"] / k["SQ_WAVE_CYCLES"], 3)
                if k.get("SQ_WAIT_ANY") is not None:
                    v["wave_wait_frac"] = round(k["SQ_WAIT_ANY"] / k["SQ_WAVE_CYCLES"], 3)
            out["valu"] = v
    return out


def main():
    args = parse()
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(relaunch_distributed(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    if args.comm_probe:
        sys.exit(comm_probe_main(args, world, rank, local_rank))
    # --comm auto: decided before this process touches the GPU (the probe children do)
    store, comm_note = None, None
    if args.comm == "auto":
        args.comm = "split"
        probe_backend = args.probe_backend or args.dist_backend
        if (world > 1 and probe_backend == "nccl") or args.probe_backend is not None:
            if world > 1:   # torch.distributed.run's store (the training process group reuses it)
                from torch.distributed.rendezvous import rendezvous
                store, _, _ = next(rendezvous("env://", rank, world))
            # the library is built ONCE, by rank 0, before any probe child starts (hipcc does not touch
            # the GPU); the others wait for it, so a cold build never runs inside a probe's timeout
            import __graft_entry__
            if rank == 0:
                __graft_entry__.build()
                if store is not None:
                    store.set("psfm_built", "1")
            elif store is not None:
                store.wait(["psfm_built"], datetime.timedelta(seconds=1800))
            probe_file = os.path.join(tempfile.gettempdir(), f"psfm_probe_{os.getpid()}.json") if rank == 0 else None
            args.comm, comm_note = choose_comm(
                store if store is not None else dist.HashStore(), rank, world,
                lambda port: launch_comm_probe(args, rank, world, local_rank, port, probe_backend, probe_file))
            if rank == 0:
                try:
                    with open(probe_file) as f:
                        probe_info = json.load(f)
                    os.remove(probe_file)
                    comm_note += (f"; probe: {probe_info['model']}, {probe_info['buckets']} buckets of "
                                  f"{probe_info['bucket_mb']} MB")
                except (OSError, ValueError, KeyError):
                    pass
            if args.dist_backend == "gloo":   # a gloo run cannot capture its collectives
                args.comm, comm_note = "split", comm_note + " (gloo run: split)"
        else:
            comm_note = "auto: split (" + ("one rank: no collective" if world == 1 else "gloo") + ")"
    if args.probe_only:
        if rank == 0:
            print(json.dumps({"comm": args.comm, "comm_note": comm_note, "world": world}), flush=True)
        return
    ndev = torch.cuda.device_count()
    if args.dist_backend == "nccl" and world > ndev:
        raise SystemExit(f"{world} ranks need {world} GPUs for RCCL, {ndev} visible "
                         f"(rehearse on fewer GPUs with --dist-backend gloo)")
    torch.cuda.set_device(local_rank % ndev)
    device = torch.device("cuda", local_rank % ndev)
    if args.dist_backend == "gloo" and args.comm != "split":
        raise SystemExit("gloo collectives cannot be captured into a HIP graph: use --comm split")
    if world == 1 and args.force_comm:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", str(_free_port()))
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=device)
    elif world > 1:
        # the store --comm auto rendezvoused on: prefixed as init_process_group's own env:// path does
        kw = dict(store=dist.PrefixStore("default_pg", store), rank=rank, world_size=world) if store is not None else {}
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=device, **kw)
        else:
            dist.init_process_group("gloo", **kw)

    import __graft_entry__
    if rank == 0 or world == 1:
        __graft_entry__.build()
    if world > 1:
        dist.barrier()
        __graft_entry__.build()
    from packnet_sfm_amd.losses import _hip_photometric as HP
    from packnet_sfm_amd.trainers.ddp_trainer import DDPTrainer, make_optimizer
    from packnet_sfm_amd.datasets.synthetic import ResidentLoader, SyntheticSfmDataset, get_datasampler

    from packnet_sfm_amd.networks.layers import fused
    kinds = {"none": set(), "all": {"bias", "bn", "gn"}}.get(args.fused_nets, set(args.fused_nets.split(",")))
    fused.FUSE.update(bias="bias" in kinds, bn="all" if "bnall" in kinds else ("resident" if "bn" in kinds else False),
                      gn="gn" in kinds)
    fused.UPCAT = not args.no_upcat
    fused.ADD_RELU = not args.no_add_relu
    fused.FORK = not args.no_fork
    fused.STEM_POOL = not args.no_stem_pool
    fused.NET_INPUTS = not args.no_net_inputs
    torch.manual_seed(0)  # identical initial weights on every rank (the trainer also broadcasts them)
    torch.backends.cudnn.benchmark = not args.no_miopen_find
    torch.backends.cudnn.deterministic = args.deterministic != "none"
    if args.deterministic == "all":
        torch.use_deterministic_algorithms(True, warn_only=True)
    model = build_model(args, device)
    model.pose_first = args.pose_first
    if not args.nchw:
        to_channels_last(model)
    opt = make_optimizer(model, 1e-4, 1e-4, capturable=not args.eager, fused=True)
    trainer = DDPTrainer(model, opt, device, amp_dtype=torch.bfloat16 if args.amp == "bf16" else None,
                         graph=not args.eager, bf16_weights=(args.amp == "bf16" and not args.eager),
                         comm=args.comm, overlap_bucket_mb=args.bucket_mb, force_comm=args.force_comm)
    images_per_step = args.batch * args.cameras
    loader = None
    if args.data_path == "sampler":
        dataset = SyntheticSfmDataset(8 * args.batch * world, args.height, args.width, N_CTX, args.cameras, seed=0)
        loader = ResidentLoader(dataset, args.batch, get_datasampler(dataset, "train"), device)
        if args.no_hip_gather:
            loader._gather_hip = lambda idx, dst: False
        batch = loader.next_into(None)
        if not args.nchw:
            net_layout(batch)
        next_batch = lambda: loader.next_into(trainer.static_batch if trainer.graphs else batch)  # noqa: E731
    elif args.data_path == "resident":
        batch = synthetic_batch(images_per_step, args.height, args.width, device, seed=rank,
                                channels_last=not args.nchw)
        next_batch = lambda: batch  # noqa: E731
    else:
        import random as _random
        from packnet_sfm_amd.datasets.augmentations import train_transforms_batch
        raw, rng = raw_frames(images_per_step, device, seed=rank), _random.Random(rank)

        def next_batch():
            b = train_transforms_batch(raw, (args.height, args.width), (0.2, 0.2, 0.2, 0.05), (), rng=rng)
            return {k: b[k] for k in ("rgb", "rgb_context", "rgb_original", "rgb_context_original", "intrinsics")}

        batch = next_batch()   # the captured (static) batch, in the nets' layout
        if not args.nchw:
            net_layout(batch)

    for i in range(args.warmup):   # the first steps include MIOpen find and the HIP-graph capture
        t_w = time.perf_counter()
        trainer.train_step(next_batch() if i else batch)
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
    host_enqueue = time.perf_counter() - t0   # host time to issue the K steps (no sync inside)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    trainer.check_finite()
    instep = k12_in_step(trainer, next_batch, device)
    batch_now = trainer.static_batch if trainer.graphs else batch
    ktimes = {} if args.no_kernel_timing else time_photometric_kernels(args, trainer, batch_now, HP)
    if world > 1:
        t = torch.tensor([elapsed], device=device, dtype=torch.float64)
        if args.dist_backend == "gloo":
            t = t.cpu()
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed = float(t)

    if rank == 0:
        images = images_per_step * world * args.steps
        value = images / elapsed
        per_step_ms = 1000.0 * elapsed / args.steps
        data = {"sampler": f"DistributedSampler(world={world}, rank) partition of a {8 * args.batch * world}-sample "
                           f"synthetic dataset resident in HBM, gathered per step",
                "resident": "one resident synthetic batch",
                "gpu-augment": "raw 375x1242 uint8 frames -> train_transforms on the GPU inside every timed step"
                }[args.data_path]
        out = {"metric": METRIC, "value": round(value, 2), "unit": "images/s", "n_gpus": world,
               "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(per_step_ms, 3),
               "host_enqueue_ms_per_step": round(1000.0 * host_enqueue / args.steps, 3),
               "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
               "dtype": "bf16" if args.amp == "bf16" else "fp32", "data": "synthetic",
               "config": {"workload": f"SelfSupModel {args.depth_net} + {args.pose_net}, {args.width}x{args.height}, "
                                      f"{args.batch} sample(s) x {args.cameras} camera(s) per GPU, 2 contexts, "
                                      f"4 full-res scales, automask min-reprojection, Adam; {args.yaml}",
                          "preset": args.config, "model": f"{args.depth_net}+{args.pose_net}",
                          "global_batch": images_per_step * world, "per_gpu_images": images_per_step,
                          "image_hw": [args.height, args.width], "parallelism": f"dp{world}",
                          "dist_backend": args.dist_backend if world > 1 else None,
                          "comm": (f"{args.comm}" + (f" ({args.bucket_mb:g} MB buckets)" if args.comm == "overlap" else "")
                                   + (" (forced at N=1)" if world == 1 else "")) if (world > 1 or args.force_comm)
                          else None, "comm_selection": comm_note, "data_path": data,
                          "net_dtype": args.amp, "loss_dtype": "fp32",
                          "net_layout": "NCHW" if args.nchw else "channels_last",
                          "step": "eager" if args.eager else "hip_graph",
                          "deterministic": args.deterministic,
                          "weights_dtype": "bf16 model + fp32 master" if (args.amp == "bf16" and not args.eager)
                          else "fp32",
                          "net_epilogues": (f"fused HIP (psfm_netops: {args.fused_nets}), the rest the reference "
                                            f"op chain" if args.fused_nets != "none" else "reference op chain"),
                          "decoder_upcat": "torch op chain" if args.no_upcat else "HIP (psfm_upcat)",
                          "weights": "random init (no network / checkpoints)", "config_key": config_key(args)}}
        out["library"] = __graft_entry__.library_hash()
        from packnet_sfm_amd import _hip as _hipmod
        out["config"]["knobs"] = _hipmod.nondefault_knobs()   # kernel-selection knobs off their defaults
        if ktimes:
            out["roofline"] = roofline(args, ktimes, instep)
        elif instep:
            out["k12_in_step"] = instep
        if world == 1 and not args.no_cpu_baseline:
            out["cpu_baseline"] = cpu_baseline(args)
        print(json.dumps(out), flush=True)
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
