"""Pinhole Camera with the reference API (packnet_sfm/geometry/camera.py:15-190):
`K`, `Tcw`, `fx/fy/cx/cy`, `Twc`, `Kinv`, `scaled`, `reconstruct`, `project`, `to`; and the
fork's FisheyeCamera (VADAS, :194-394): intrinsics dict {k [B,7], s, div, ux, uy}, `Tcw`,
`image_size`, `reconstruct`, `project` (+ `scaled`, the per-scale intrinsics of the loss).

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


_FLT_EPS = 2.220446049250313e-16  # sys.float_info.epsilon (camera.py:281, :352, :365)


class FisheyeCamera(nn.Module):
    """VADAS fisheye camera (geometry/camera.py:194-394).  reconstruct keeps the reference's
    theta ~= r_d approximation (:276-286); project's frame='w' applies Tcw to the points as
    R X + t (the fork's `Pose @ [B,3,N]` raises)."""

    def __init__(self, intrinsics, Tcw=None, image_size=None):
        super().__init__()
        self.k, self.s, self.div = intrinsics["k"], intrinsics["s"], intrinsics["div"]
        self.ux, self.uy = intrinsics["ux"], intrinsics["uy"]
        self.Tcw = Pose.identity(len(self.k), device=self.k.device, dtype=self.k.dtype) if Tcw is None else Tcw
        self.image_size = image_size

    def __len__(self):
        return len(self.k)

    @property
    def intrinsics(self):
        return {"k": self.k, "s": self.s, "div": self.div, "ux": self.ux, "uy": self.uy}

    def to(self, *args, **kwargs):
        for n in ("k", "s", "div", "ux", "uy"):
            setattr(self, n, getattr(self, n).to(*args, **kwargs))
        self.Tcw = self.Tcw.to(*args, **kwargs)
        return self

    @property
    def Twc(self):
        return self.Tcw.inverse()

    def scaled(self, x_scale, y_scale=None):
        """Centre scaled as (c + 0.5) s - 0.5; k, s, div unchanged (multiview_photometric_loss.py:166-186)."""
        y_scale = x_scale if y_scale is None else y_scale
        size = None if self.image_size is None else (round(self.image_size[0] * y_scale),
                                                     round(self.image_size[1] * x_scale))
        return FisheyeCamera({"k": self.k, "s": self.s, "div": self.div, "ux": (self.ux + 0.5) * x_scale - 0.5,
                              "uy": (self.uy + 0.5) * y_scale - 0.5}, Tcw=self.Tcw, image_size=size)

    def reconstruct(self, depth, frame="w"):
        B, C, H, W = depth.shape
        assert C == 1
        grid = image_grid(B, H, W, depth.dtype, depth.device, normalized=False).view(B, 3, -1)
        xd = (grid[:, 0] - self.ux.unsqueeze(1)) / self.s.unsqueeze(1)
        yd = (grid[:, 1] - self.uy.unsqueeze(1)) / self.div.unsqueeze(1)
        rd = torch.sqrt(xd ** 2 + yd ** 2)
        r = torch.tan(rd)
        rds = torch.where(rd < _FLT_EPS, torch.full_like(rd, _FLT_EPS), rd)
        d = depth.view(B, -1)
        Xc = torch.stack([(r / rds) * xd * d, (r / rds) * yd * d, d], 1).view(B, 3, H, W)
        if frame == "c":
            return Xc
        if frame == "w":
            return self.Twc @ Xc
        raise ValueError("Unknown reference frame {}".format(frame))

    def project(self, X, frame="w"):
        if X.dim() == 4:
            B, C, H, W = X.shape
        elif X.dim() == 3:
            B, C, N = X.shape
            if self.image_size is None:
                raise ValueError("image_size must be provided for 3D point cloud projection.")
            H, W = self.image_size
        else:
            raise ValueError("Input X must be of shape [B,3,H,W] or [B,3,N]")
        assert C == 3
        Xf = X.reshape(B, 3, -1)
        if frame == "w":
            m = self.Tcw.mat
            Xf = m[:, :3, :3].bmm(Xf) + m[:, :3, 3:]
        elif frame != "c":
            raise ValueError("Unknown reference frame {}".format(frame))
        Z = Xf[:, 2].clamp(min=_FLT_EPS)
        xn, yn = Xf[:, 0] / Z, Xf[:, 1] / Z
        r = torch.sqrt(xn ** 2 + yn ** 2)
        th = torch.atan(r)
        poly = self.k[:, 0].unsqueeze(1)
        for i in range(1, 7):
            poly = poly + self.k[:, i].unsqueeze(1) * torch.pow(th, i)
        rs = torch.where(r < _FLT_EPS, torch.full_like(r, _FLT_EPS), r)
        u = self.s.unsqueeze(1) * ((poly / rs) * xn) + self.ux.unsqueeze(1)
        v = self.div.unsqueeze(1) * ((poly / rs) * yn) + self.uy.unsqueeze(1)
        coords = torch.stack([2 * u / (W - 1) - 1.0, 2 * v / (H - 1) - 1.0], -1)
        return coords.view(B, H, W, 2) if X.dim() == 4 else coords
