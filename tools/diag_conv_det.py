"""Run-to-run spread of MIOpen conv gradients (bf16 channels_last vs fp32) on ResNet-SAN layer
shapes, and of the whole ResNetSAN01+PoseNet backward, with and without deterministic algorithms."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

dev = torch.device("cuda:0")
torch.backends.cudnn.benchmark = False


def rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-30))


def conv_case(cin, cout, k, stride, H, W, dtype, B=2):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, cin, H, W, device=dev, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(cout, cin, k, k, device=dev, generator=g) * 0.05).to(dtype)
    w = torch.empty_like(w, memory_format=torch.channels_last).copy_(w)
    gy = None
    res = []
    for _ in range(3):
        xx, ww = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
        y = F.conv2d(xx, ww, None, stride, k // 2)
        if gy is None:
            gy = torch.randn(y.shape, device=dev, generator=g).to(dtype).contiguous(memory_format=torch.channels_last)
        y.backward(gy)
        res.append((xx.grad.clone(), ww.grad.clone()))
    # fp64 CPU reference of the same bf16-valued operands
    xd, wd = x.double().cpu().requires_grad_(True), w.double().cpu().requires_grad_(True)
    F.conv2d(xd, wd, None, stride, k // 2).backward(gy.double().cpu())
    return [rel(res[1][0], res[0][0]), rel(res[2][1], res[0][1]), rel(res[0][0].cpu(), xd.grad),
            rel(res[0][1].cpu(), wd.grad)]


for det in (False, True):
    torch.use_deterministic_algorithms(det, warn_only=True)
    for dtype in (torch.bfloat16, torch.float32):
        for shp in ((64, 64, 3, 1, 48, 160), (128, 256, 3, 2, 24, 80), (256, 512, 3, 2, 12, 40),
                    (512, 512, 3, 1, 6, 20), (3, 64, 7, 2, 192, 640)):
            r = conv_case(*shp, dtype)
            print(f"det={det} {str(dtype)[6:]:8s} conv{shp}: run-to-run dgrad {r[0]:.2e} wgrad {r[1]:.2e} | "
                  f"vs fp64 dgrad {r[2]:.2e} wgrad {r[3]:.2e}", flush=True)
