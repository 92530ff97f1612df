"""GPU check + timing of the composed PackNet packing layer (packconv.py, include/psfm_packconv.h).

  python tools/pc_check.py [--big] [--time] [--iters N]

Parity: the HIP composed forward / backward against the reference chain
packing -> Conv3d -> view -> ConstantPad2d -> Conv2d (layers01.py:239-246, :34-39) evaluated on the
same bf16-rounded inputs, in float64 on the CPU (small shapes) or float32 on the GPU (--big: the
benchmarked PackNet01 / PackNetSAN01 first-layer shapes).  Timing: the composed path vs the round-4
path (fused pack3d kernel + MIOpen Conv2d) under bf16 autocast, fwd and fwd+bwd, HIP events."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import packnet_sfm_amd  # noqa: E402,F401
from packnet_sfm_amd.networks.layers.packnet import packconv  # noqa: E402
from packnet_sfm_amd.networks.layers.packnet.layers01 import PackLayerConv3d, packing  # noqa: E402
from packnet_sfm_amd.networks.layers.packnet.pack3d import pack_conv3d  # noqa: E402


def chain(x, W2, w3, b3, k):
    V = F.conv3d(packing(x).unsqueeze(1), w3, b3, padding=1)
    B, d, Kp, Ho, Wo = V.shape
    return F.conv2d(F.pad(V.reshape(B, d * Kp, Ho, Wo), [k // 2] * 4), W2)


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).abs().max() / b.abs().max().clamp(min=1e-30)), float((a - b).norm() / b.norm().clamp(min=1e-30))


def case(B, C, H, W, d, k, ref_dev, seed=0, bias_scale=0.3):
    g = torch.Generator().manual_seed(seed)
    bf = torch.bfloat16
    x = torch.randn(B, C, H, W, generator=g).to(bf)
    W2 = (torch.randn(C, 4 * C * d, k, k, generator=g) / (4 * C * d * k * k) ** 0.5).to(bf)
    w3 = (torch.randn(d, 1, 3, 3, 3, generator=g) / 27 ** 0.5).to(bf)
    b3 = (bias_scale * torch.randn(d, generator=g)).to(bf)
    gy = torch.randn(B, C, H // 2, W // 2, generator=g).to(bf)
    # HIP
    conv3d = torch.nn.Conv3d(1, d, 3, padding=1).cuda()
    conv2d = torch.nn.Conv2d(4 * C * d, C, k).cuda()
    with torch.no_grad():
        conv3d.weight.copy_(w3.float())
        conv3d.bias.copy_(b3.float())
        conv2d.weight.copy_(W2.float())
    xd = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = packconv.pack_conv2d(xd, conv3d, conv2d, k)
    y.backward(gy.cuda().contiguous(memory_format=torch.channels_last))
    torch.cuda.synchronize()
    # reference chain on the same bf16 values
    dt = torch.float64 if ref_dev == "cpu" else torch.float32
    xr = x.to(ref_dev, dt).requires_grad_(True)
    W2r, w3r, b3r = (t.to(ref_dev, dt).requires_grad_(True) for t in (W2, w3, b3))
    yr = chain(xr, W2r, w3r, b3r, k)
    yr.backward(gy.to(ref_dev, dt))
    res = {"y": rel(y.detach(), yr.detach()), "dx": rel(xd.grad, xr.grad), "dW2": rel(conv2d.weight.grad, W2r.grad),
           "dw3": rel(conv3d.weight.grad, w3r.grad), "db3": rel(conv3d.bias.grad, b3r.grad)}
    return res


def timeit(fn, iters):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(iters):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    ts.sort()
    return ts[len(ts) // 2]


def bench(B, C, H, W, d, k, iters):
    torch.manual_seed(0)
    m = PackLayerConv3d(C, k, d=d).cuda()
    x = torch.randn(B, C, H, W, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    gy = torch.randn(B, C, H // 2, W // 2, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    c = m.conv

    def old_f():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return F.conv2d(pack_conv3d(x, m.conv3d, 2, m.pack), c.conv_base.weight, None, 1, k // 2)

    def new_f():
        with torch.autocast("cuda", dtype=torch.bfloat16):
            return packconv.pack_conv2d(x, m.conv3d, c.conv_base, k)

    out = {}
    for name, f in (("round4", old_f), ("composed", new_f)):
        tf = timeit(lambda: f(), iters)
        tb = timeit(lambda: torch.autograd.backward(f(), gy), iters)
        out[name] = (tf, tb)
    return out


def _heartbeat():
    import threading

    def beat():
        t0 = time.time()
        while True:
            time.sleep(20)
            print(f"  ... {time.time() - t0:.0f}s", flush=True)
    threading.Thread(target=beat, daemon=True).start()


def main():
    _heartbeat()
    ap = argparse.ArgumentParser()
    ap.add_argument("--big", action="store_true")
    ap.add_argument("--time", action="store_true")
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--shapes", default=None, help="B,C,H,W,d,k;... (timing)")
    a = ap.parse_args()
    torch.backends.cudnn.benchmark = True
    small = [(2, 32, 16, 24, 4, 3), (2, 64, 20, 28, 8, 5), (1, 32, 14, 18, 8, 5), (2, 64, 12, 16, 4, 3),
             (1, 96, 16, 144, 8, 3), (3, 128, 10, 12, 8, 3)]
    t0 = time.time()
    for s in (small if not a.time else []):
        r = case(*s, ref_dev="cpu")
        print("small", s, {k_: f"{v[0]:.2e}/{v[1]:.2e}" for k_, v in r.items()}, flush=True)
    if a.big:
        for s in [(6, 64, 192, 640, 8, 5), (4, 32, 384, 640, 4, 5), (6, 64, 96, 320, 8, 3), (6, 512, 12, 40, 8, 3)]:
            r = case(*s, ref_dev="cuda")
            print("big", s, {k_: f"{v[0]:.2e}/{v[1]:.2e}" for k_, v in r.items()}, flush=True)
    if a.time:
        shapes = ([tuple(int(v) for v in t.split(",")) for t in a.shapes.split(";")] if a.shapes else
                  [(6, 64, 192, 640, 8, 5), (6, 64, 96, 320, 8, 3), (6, 128, 48, 160, 8, 3), (6, 256, 24, 80, 8, 3),
                   (6, 512, 12, 40, 8, 3), (4, 32, 384, 640, 4, 5)])
        for s in shapes:
            r = bench(*s, a.iters)
            print("time", s, {k_: f"fwd {v[0] * 1e3:.0f} us, fwd+bwd {v[1] * 1e3:.0f} us" for k_, v in r.items()},
                  flush=True)
    print(f"done in {time.time() - t0:.1f}s")


if __name__ == "__main__":
    main()
