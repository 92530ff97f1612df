"""Progress-printing probe of the composed packing layer at PackNet shapes: HIP fwd / bwd timing
(HIP events), then the fp32 torch chain on the same device (MIOpen) for comparison."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402

from packnet_sfm_amd.networks.layers.packnet import packconv  # noqa: E402
from oracle.packconv_oracle import chain  # noqa: E402


def ev_time(fn, n=5):
    ts = []
    for _ in range(n):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        fn()
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b) * 1e3)
    return sorted(ts)[n // 2]


def main():
    ref = "--ref" in sys.argv
    shapes = [(6, 64, 192, 640, 8, 5), (6, 64, 96, 320, 8, 3), (6, 128, 48, 160, 8, 3), (6, 256, 24, 80, 8, 3),
              (6, 512, 12, 40, 8, 3), (4, 32, 384, 640, 4, 5)]
    for (B, C, H, W, d, k) in shapes:
        t0 = time.time()
        g = torch.Generator().manual_seed(0)
        x = torch.randn(B, C, H, W, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=torch.channels_last)
        W2 = (torch.randn(C, 4 * C * d, k, k, generator=g) / (4 * C * d * k * k) ** 0.5).cuda().requires_grad_(True)
        w3 = (torch.randn(d, 1, 3, 3, 3, generator=g) / 27 ** 0.5).cuda().requires_grad_(True)
        b3 = (0.3 * torch.randn(d, generator=g)).cuda().requires_grad_(True)
        gy = torch.randn(B, C, H // 2, W // 2, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        y = packconv.PackConvFn.apply(x, W2, w3, b3, k)
        torch.cuda.synchronize()
        print(f"{(B, C, H, W, d, k)} first fwd done {time.time() - t0:.1f}s", flush=True)
        y.backward(gy)
        torch.cuda.synchronize()
        print(f"  first bwd done {time.time() - t0:.1f}s", flush=True)
        tf = ev_time(lambda: packconv.PackConvFn.apply(x, W2, w3, b3, k))
        tb = ev_time(lambda: packconv.PackConvFn.apply(x, W2, w3, b3, k).backward(gy))
        print(f"  HIP fwd {tf:.0f} us  fwd+bwd {tb:.0f} us", flush=True)
        if ref:
            xr, W2r, w3r, b3r = (t.detach().float().to(torch.bfloat16).float().requires_grad_(True) for t in (x, W2, w3, b3))
            yr = chain(xr, W2r, w3r, b3r, k)
            yr.backward(gy.float())
            torch.cuda.synchronize()
            print(f"  fp32 chain done {time.time() - t0:.1f}s", flush=True)
            for n, a, b in (("y", y.float(), yr), ("dx", x.grad.float(), xr.grad)):
                print(f"  {n} rel l2 {float((a - b).norm() / b.norm()):.2e} max {float((a - b).abs().max() / b.abs().max()):.2e}",
                      flush=True)


if __name__ == "__main__":
    main()
