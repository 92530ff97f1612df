"""Per-tensor comparison of the HIP composed-layer outputs (y, dx, dWeff, dU, dCorner, dBT) with a
float64 CPU autograd of the same decomposition (tests/test_packconv.py composed form)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))
import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import packnet_sfm_amd  # noqa: E402,F401
from packnet_sfm_amd.networks.layers.packnet import packconv  # noqa: E402
from packnet_sfm_amd.networks.layers.packnet.layers01 import packing  # noqa: E402


def composed(x, Weff, U, Cn, bt, k):
    C = Weff.shape[0]
    pk, pe, ke = k // 2, k // 2 + 1, k + 2
    P = packing(x)
    B, Kp, Ho, Wo = P.shape
    y = F.conv2d(P, Weff, padding=pe)
    rc = lambda n: torch.tensor([i if i < pk else (2 * pk - (n - 1 - i) if i >= n - pk else pk) for i in range(n)])
    y = y + bt[rc(Ho)][:, rc(Wo)].permute(2, 0, 1)
    lines = [P[:, :, 0, :], P[:, :, Ho - 1, :], P[:, :, :, 0], P[:, :, :, Wo - 1]]
    E = [F.conv1d(l_, U[e].reshape(pk * C, Kp, ke), padding=pe).reshape(B, pk, C, -1) for e, l_ in enumerate(lines)]
    corr = torch.zeros_like(y)
    corr[:, :, :pk, :] += E[0].flip(1).permute(0, 2, 1, 3)
    corr[:, :, Ho - pk:, :] += E[1].flip(1).permute(0, 2, 1, 3)
    corr[:, :, :, :pk] += E[2].flip(1).permute(0, 2, 3, 1)
    corr[:, :, :, Wo - pk:] += E[3].flip(1).permute(0, 2, 3, 1)
    px = [P[:, :, 0, 0], P[:, :, Ho - 1, 0], P[:, :, 0, Wo - 1], P[:, :, Ho - 1, Wo - 1]]
    cf = torch.zeros_like(y)
    for cn in range(4):
        v = torch.einsum("ijmk,bk->bmij", Cn[cn], px[cn]).flip(2, 3)
        ys = slice(0, pk) if cn % 2 == 0 else slice(Ho - pk, Ho)
        xs = slice(0, pk) if cn < 2 else slice(Wo - pk, Wo)
        cf[:, :, ys, xs] = cf[:, :, ys, xs] + v
    return y - corr + cf


def run(B, C, H, W, d, k, seed=0):
    g = torch.Generator().manual_seed(seed)
    bf = torch.bfloat16
    x = torch.randn(B, C, H, W, generator=g).to(bf)
    W2 = (torch.randn(C, 4 * C * d, k, k, generator=g) / (4 * C * d * k * k) ** 0.5).to(bf)
    w3 = (torch.randn(d, 1, 3, 3, 3, generator=g) / 27 ** 0.5).to(bf)
    b3 = (0.3 * torch.randn(d, generator=g)).to(bf)
    gy = torch.randn(B, C, H // 2, W // 2, generator=g).to(bf)
    Weff, U, Cn, bt = packconv.compose(W2.float(), w3.float(), b3.float(), k)
    # round the weights the kernels use to bf16 so both sides see the same operands
    Weffb, Ub = Weff.to(bf).float(), U.to(bf).float()
    ins = [t.clone().cuda().requires_grad_(True) for t in (Weffb, Ub, Cn, bt)]
    xd = x.cuda().contiguous(memory_format=torch.channels_last).requires_grad_(True)
    y = packconv.PackConvFn.apply(xd, *ins, k)
    y.backward(gy.cuda().contiguous(memory_format=torch.channels_last))
    ref = [t.double().requires_grad_(True) for t in (Weffb, Ub, Cn, bt)]
    xr = x.double().requires_grad_(True)
    yr = composed(xr, *ref, k)
    yr.backward(gy.double())
    out = {}
    for n, a, b in [("y", y.detach(), yr.detach()), ("dx", xd.grad, xr.grad)] + \
            [(n, t.grad, r.grad) for n, t, r in zip(("dWeff", "dU", "dCn", "dbt"), ins, ref)]:
        a, b = a.double().cpu(), b.double().cpu()
        err = (a - b).abs()
        out[n] = f"max {float(err.max() / b.abs().max()):.2e} l2 {float((a - b).norm() / b.norm()):.2e}"
        if n in ("dU", "dCn", "dbt"):
            # per leading index
            out[n] += " per-slice " + " ".join(f"{float(err[i].max() / b.abs().max()):.1e}" for i in range(a.shape[0]))
    print((B, C, H, W, d, k), out, flush=True)


if __name__ == "__main__":
    for s in [(2, 32, 16, 24, 4, 3), (2, 64, 20, 28, 8, 5), (1, 32, 14, 18, 8, 5), (1, 96, 16, 144, 8, 3),
              (3, 128, 10, 12, 8, 3)]:
        run(*s)
