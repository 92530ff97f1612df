"""Which kernels ATen launches for nn.BatchNorm2d (train) on channels_last bf16 activations of the
ResNet stem / layer1 / layer2 shapes (forward + backward), by torch.profiler: are there layout copies
around MIOpen's BatchNorm?  python tools/diag_bn_layout.py"""
import os
import sys

import torch
import torch.nn as nn
from torch.profiler import ProfilerActivity, profile

dev = torch.device("cuda")
print("PYTORCH_MIOPEN_SUGGEST_NHWC_BATCHNORM =", os.environ.get("PYTORCH_MIOPEN_SUGGEST_NHWC_BATCHNORM"), flush=True)
for shape in ((4, 64, 96, 320), (4, 64, 48, 160), (4, 128, 24, 80)):
    bn = nn.BatchNorm2d(shape[1]).to(dev).train()
    x = torch.randn(shape, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x.requires_grad_(True)
    for _ in range(2):
        y = bn(x)
        y.backward(torch.ones_like(y))
    torch.cuda.synchronize()
    with profile(activities=[ProfilerActivity.CUDA]) as prof:
        y = bn(x)
        y.backward(torch.ones_like(y))
        torch.cuda.synchronize()
    print(shape, "y channels_last:", y.is_contiguous(memory_format=torch.channels_last),
          "dx channels_last:", x.grad.is_contiguous(memory_format=torch.channels_last), flush=True)
    for e in prof.key_averages():
        if e.device_type is not None and "CUDA" in str(e.device_type) or getattr(e, "device_time_total", 0) > 0:
            print(f"   {e.count:3d} x {e.device_time_total / max(e.count, 1):8.1f} us  {e.key[:110]}")
sys.stdout.flush()
