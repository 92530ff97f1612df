#!/usr/bin/env python3
"""Which forward-only calls survive HIP-graph capture?  (tools/gn_bench.py's
capture of repeated forward-only GroupNorm calls crashed in capture_end.)

One case per process (run them chained with &&, the likely crash last): 3 calls of a forward
captured into one graph, replayed, compared with eager.  Cases cross the op (the fused
psfm_gn_act / torch's own group_norm chain) with grad mode (no_grad / grad enabled with the
GroupNorm affine parameters requiring grad, the outputs discarded, or kept alive: _keep).
  python tools/diag_capture_fwd.py CASE [ITERS [N C H W]]   (default 3 calls, [4, 64, 48, 160], ELU;
  any other shape: ReLU, as PoseNet's conv_gn — tools/gn_bench.py's r3d crash was 20 calls of
  [4, 16, 96, 320] with grad enabled)
"""
import os
import sys

CASES = ["fused_nograd", "fused_grad", "torch_nograd", "torch_grad", "fused_grad_keep"]


def child(case, iters=3, shape=(4, 64, 48, 160)):
    import torch
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import __graft_entry__
    __graft_entry__.build()
    from packnet_sfm_amd.networks.layers import fused as FU
    dev = torch.device("cuda:0")
    C = shape[1]
    act = FU.ACT_ELU if tuple(shape) == (4, 64, 48, 160) else FU.ACT_RELU
    gn = torch.nn.GroupNorm(16, C).to(dev)
    x = torch.randn(*shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = torch.randn(C, device=dev)
    fn = torch.nn.functional.elu if act == FU.ACT_ELU else torch.relu
    if case.startswith("fused"):
        call = lambda: FU.gn_act(x, b, gn, act=act)  # noqa: E731
    else:
        call = lambda: fn(gn(x.float() + b.view(1, -1, 1, 1)))  # noqa: E731
    grad = "nograd" not in case
    keep = []
    with torch.set_grad_enabled(grad):
        ref = call().detach().clone()
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            call()
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            outs = []
            for _ in range(iters):
                y = call()
                outs.append(y.detach())
                if case.endswith("keep"):
                    keep.append(y)        # the autograd graph stays alive past the capture
        g.replay()
        torch.cuda.synchronize()
    ok = all(torch.equal(o, ref) for o in outs)
    print(f"{case}: captured and replayed, outputs equal eager: {ok}", flush=True)
    return 0 if ok else 1


if __name__ == "__main__":
    assert len(sys.argv) in (2, 3, 7) and sys.argv[1] in CASES, CASES
    it = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    shp = tuple(int(v) for v in sys.argv[3:7]) if len(sys.argv) == 7 else (4, 64, 48, 160)
    sys.exit(child(sys.argv[1], it, shp))
