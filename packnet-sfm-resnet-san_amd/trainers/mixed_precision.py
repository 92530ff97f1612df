"""bf16 model weights with fp32 master weights in the optimizer.

Numerically the same forward/backward as `torch.autocast(bfloat16)` (which re-casts every fp32
conv weight to bf16 on every forward and casts its gradient back): conv/linear weights are
stored as bf16 = round(master), gradients arrive in bf16 and are widened exactly into fp32
master gradients.  Cost per step: one foreach copy in, one foreach copy out — instead of ~200
cast kernels.  Normalisation parameters stay fp32.
"""
import torch
import torch.nn as nn

_LOWP_MODULES = (nn.Conv1d, nn.Conv2d, nn.Conv3d, nn.ConvTranspose2d, nn.Linear)


class Bf16MasterWeights:
    def __init__(self, model, optimizer, dtype=torch.bfloat16):
        self.lp, self.master = [], []
        for m in model.modules():
            if isinstance(m, _LOWP_MODULES):
                for p in m.parameters(recurse=False):
                    if p.requires_grad and p.dtype == torch.float32:
                        master = p.detach().clone()
                        p.data = p.data.to(dtype)
                        self.lp.append(p)
                        self.master.append(master)
        idmap = {id(p): mp for p, mp in zip(self.lp, self.master)}
        assert not optimizer.state, "swap parameters before the first optimizer step"
        for g in optimizer.param_groups:
            g["params"] = [idmap.get(id(p), p) for p in g["params"]]
        for mp in self.master:
            mp.grad = torch.zeros_like(mp)

    @torch.no_grad()
    def grads_to_master(self):
        """Widen the bf16 gradients into the fp32 master gradients (exact)."""
        pairs = [(mp.grad, p.grad) for mp, p in zip(self.master, self.lp) if p.grad is not None]
        if pairs:
            torch._foreach_copy_([a for a, _ in pairs], [b for _, b in pairs])

    @torch.no_grad()
    def master_to_model(self):
        torch._foreach_copy_(self.lp, self.master)
