"""Pinhole Camera with the reference API (packnet_sfm/geometry/camera.py:15-190):
`K`, `Tcw`, `fx/fy/cx/cy`, `Twc`, `Kinv`, `scaled`, `reconstruct`, `project`, `to`.

`reconstruct`/`project` are the reference's standalone point-cloud API and are
elementwise [B,3,H,W] tensor algebra (kept in torch); the hot path never calls them — the
loss and `view_synthesis` run the fused HIP kernel instead.
"""
import torch
import torch.nn as nn

from .camera_utils import pinhole_inverse, scale_intrinsics
from .pose import Pose
from ..utils.image import image_grid


class Camera(nn.Module):
    def __init__(self, K, Tcw=None):
        super().__init__()
        self.K = K
        self.Tcw = Pose.identity(len(K), device=K.device, dtype=K.dtype) if Tcw is None else Tcw

    def __len__(self):
        return len(self.K)

    def to(self, *args, **kwargs):
        self.K = self.K.to(*args, **kwargs)
        self.Tcw = self.Tcw.to(*args, **kwargs)
        return self

    @property
    def fx(self):
        return self.K[:, 0, 0]

    @property
    def fy(self):
        return self.K[:, 1, 1]

    @property
    def cx(self):
        return self.K[:, 0, 2]

    @property
    def cy(self):
        return self.K[:, 1, 2]

    @property
    def Twc(self):
        return self.Tcw.inverse()

    @property
    def Kinv(self):
        return pinhole_inverse(self.K)

    def scaled(self, x_scale, y_scale=None):
        if y_scale is None:
            y_scale = x_scale
        if x_scale == 1.0 and y_scale == 1.0:
            return self
        return Camera(scale_intrinsics(self.K.clone(), x_scale, y_scale), Tcw=self.Tcw)

    def reconstruct(self, depth, frame="w"):
        """Pixel-wise 3D points [B,3,H,W] from depth [B,1,H,W]."""
        B, C, H, W = depth.shape
        assert C == 1
        grid = image_grid(B, H, W, depth.dtype, depth.device, normalized=False).view(B, 3, -1)
        Xc = self.Kinv.bmm(grid).view(B, 3, H, W) * depth
        if frame == "c":
            return Xc
        if frame == "w":
            return self.Twc @ Xc
        raise ValueError("Unknown reference frame {}".format(frame))

    def project(self, X, frame="w"):
        """Normalised sampling grid [B,H,W,2] of points X [B,3,H,W]."""
        B, C, H, W = X.shape
        assert C == 3
        if frame == "c":
            Xc = self.K.bmm(X.view(B, 3, -1))
        elif frame == "w":
            Xc = self.K.bmm((self.Tcw @ X).view(B, 3, -1))
        else:
            raise ValueError("Unknown reference frame {}".format(frame))
        Z = Xc[:, 2].clamp(min=1e-5)
        Xn = 2 * (Xc[:, 0] / Z) / (W - 1) - 1.0
        Yn = 2 * (Xc[:, 1] / Z) / (H - 1) - 1.0
        return torch.stack([Xn, Yn], dim=-1).view(B, H, W, 2)
