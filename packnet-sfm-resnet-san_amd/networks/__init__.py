"""Depth and pose networks (PyTorch-ROCm / MIOpen), registry by reference class name."""


def load_depth_net(name, **kwargs):
    from .depth.DepthResNet import DepthResNet
    from .depth.PackNet01 import PackNet01
    from .depth.PackNetSAN01 import PackNetSAN01
    from .depth.ResNetSAN01 import ResNetSAN01
    nets = {"DepthResNet": DepthResNet, "PackNet01": PackNet01, "PackNetSAN01": PackNetSAN01,
            "ResNetSAN01": ResNetSAN01}
    if name not in nets:
        raise ValueError(f"depth net {name} is not provided (available: {sorted(nets)})")
    return nets[name](**kwargs)


def load_pose_net(name, **kwargs):
    from .pose.PoseNet import PoseNet
    from .pose.PoseResNet import PoseResNet
    nets = {"PoseNet": PoseNet, "PoseResNet": PoseResNet}
    if name not in nets:
        raise ValueError(f"pose net {name} is not provided (available: {sorted(nets)})")
    return nets[name](**kwargs)
