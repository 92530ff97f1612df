"""Camera helpers and `view_synthesis`.

Mirrors packnet_sfm/geometry/camera_utils.py: `construct_K` (:9-13), `scale_intrinsics`
(:16-22), `view_synthesis` (:27-59).  `view_synthesis` runs the fused HIP warp kernel
(lift -> transform -> project -> bilinear gather in one pass, no [B,3,H,W] point cloud or
[B,H,W,2] grid materialised); the reference's ATen chain is restated only in oracle/.
"""
import torch


def construct_K(fx, fy, cx, cy, dtype=torch.float, device=None):
    return torch.tensor([[fx, 0, cx], [0, fy, cy], [0, 0, 1]], dtype=dtype, device=device)


def scale_intrinsics(K, x_scale, y_scale):
    """In place, like the reference: focal lengths scale, principal point (c+0.5)s-0.5."""
    K[..., 0, 0] *= x_scale
    K[..., 1, 1] *= y_scale
    K[..., 0, 2] = (K[..., 0, 2] + 0.5) * x_scale - 0.5
    K[..., 1, 2] = (K[..., 1, 2] + 0.5) * y_scale - 0.5
    return K


def pinhole_inverse(K):
    """Closed-form K^-1 of camera.py:72-81 (the clone keeps K's other entries, incl. skew)."""
    Ki = K.clone()
    Ki[:, 0, 0] = 1.0 / K[:, 0, 0]
    Ki[:, 1, 1] = 1.0 / K[:, 1, 1]
    Ki[:, 0, 2] = -1.0 * K[:, 0, 2] / K[:, 0, 0]
    Ki[:, 1, 2] = -1.0 * K[:, 1, 2] / K[:, 1, 1]
    return Ki


def view_synthesis(ref_image, depth, ref_cam, cam, mode="bilinear", padding_mode="zeros"):
    """Warp `ref_image` [B,3,H,W] into `cam`'s view using `depth` [B,1,H,W]
    (bilinear, zero padding, align_corners=True).  Differentiable w.r.t. depth and the poses.
    `Camera` (pinhole) or `FisheyeCamera` (VADAS) pairs."""
    if mode != "bilinear" or padding_mode != "zeros":
        raise NotImplementedError("HIP view_synthesis implements bilinear / zeros (reference default)")
    assert depth.size(1) == 1
    from .. import _hip
    from ..losses._hip_photometric import ViewSynthesisFn
    from .camera import FisheyeCamera
    # world->ref composite: ref_cam.Tcw @ cam.Twc (camera.py:144 then :165)
    T = ref_cam.Tcw.mat.bmm(cam.Twc.mat)[:, :3, :]
    B = depth.shape[0]
    if isinstance(cam, FisheyeCamera) != isinstance(ref_cam, FisheyeCamera):
        raise ValueError("view_synthesis: both cameras pinhole or both fisheye")
    if isinstance(cam, FisheyeCamera):
        f = lambda t: t.float().reshape(B, -1)  # noqa: E731
        rec = torch.cat([f(cam.s), f(cam.div), f(cam.ux), f(cam.uy), f(ref_cam.k), f(ref_cam.s), f(ref_cam.div),
                         f(ref_cam.ux), f(ref_cam.uy), torch.zeros(B, 3, device=depth.device)], -1)
        return ViewSynthesisFn.apply(ref_image, depth, rec, T, _hip.CAM_FISHEYE)
    rec = torch.cat([pinhole_inverse(cam.K.float()).reshape(B, 9), ref_cam.K.float().reshape(B, 9)], -1)
    return ViewSynthesisFn.apply(ref_image, depth, rec, T, _hip.CAM_PINHOLE)
