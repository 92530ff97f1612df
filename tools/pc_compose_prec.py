import os, sys
sys.path.insert(0, '/root/repo')
import torch
import packnet_sfm_amd
from packnet_sfm_amd.networks.layers.packnet import packconv
torch.manual_seed(0)
for C, d, k in [(32, 4, 3), (64, 8, 5)]:
    W2 = torch.randn(C, 4*C*d, k, k) / (4*C*d*k*k) ** 0.5
    w3 = torch.randn(d, 1, 3, 3, 3) / 27 ** 0.5
    b3 = 0.3 * torch.randn(d)
    outs_c = packconv.compose(*(t.double().requires_grad_(True) for t in (W2, w3, b3)), k)
    gs = [torch.randn_like(o) for o in outs_c]
    for mode in ["default", "no_tf32", "no_cudnn"]:
        if mode == "no_tf32":
            torch.backends.cudnn.allow_tf32 = False
        ins = [t.cuda().requires_grad_(True) for t in (W2, w3, b3)]
        ctx = torch.backends.cudnn.flags(enabled=False) if mode == "no_cudnn" else torch.backends.cudnn.flags(enabled=True)
        with ctx:
            outs = packconv.compose(*ins, k)
            gr = torch.autograd.grad(outs, ins, [g.float().cuda() for g in gs])
        insc = [t.double().requires_grad_(True) for t in (W2, w3, b3)]
        outc = packconv.compose(*insc, k)
        grc = torch.autograd.grad(outc, insc, gs)
        fe = [float((a.double().cpu()-b).abs().max()/b.abs().max()) for a, b in zip(outs, outc)]
        ge = [float((a.double().cpu()-b).abs().max()/b.abs().max()) for a, b in zip(gr, grc)]
        print(C, d, k, mode, 'fwd', ['%.1e' % e for e in fe], 'bwd', ['%.1e' % e for e in ge], flush=True)
        torch.backends.cudnn.allow_tf32 = True
# timing of compose fwd+bwd at the first layer
import time
C, d, k = 64, 8, 5
W2 = torch.randn(C, 4*C*d, k, k, device='cuda', requires_grad=True); w3 = torch.randn(d,1,3,3,3, device='cuda', requires_grad=True); b3 = torch.randn(d, device='cuda', requires_grad=True)
for mode in ["default", "no_cudnn"]:
    ctx = torch.backends.cudnn.flags(enabled=False) if mode == "no_cudnn" else torch.backends.cudnn.flags(enabled=True)
    with ctx:
        for it in range(5):
            torch.cuda.synchronize(); t0 = time.time()
            outs = packconv.compose(W2, w3, b3, k)
            torch.cuda.synchronize(); t1 = time.time()
            torch.autograd.backward(outs, [torch.ones_like(o) for o in outs])
            torch.cuda.synchronize(); t2 = time.time()
        print(mode, 'compose fwd %.0f us bwd %.0f us' % ((t1-t0)*1e6, (t2-t1)*1e6), flush=True)
