"""FisheyeCamera (VADAS) API of the build (geometry/camera.py) against the reference's own
fisheye reconstruct / project (golden tests/golden/fisheye_small.npz, tools/gen_goldens.py).
CPU: the camera classes are the reference's tensor API (torch), not the hot path."""
import numpy as np
import torch

import golden_util as gu


def _T(a):
    return torch.from_numpy(np.ascontiguousarray(a))


def _intr(z):
    return {k: _T(z[f"intr_{k}"]) for k in ("k", "s", "div", "ux", "uy")}


def test_reconstruct_and_project_match_reference():
    from packnet_sfm_amd.geometry.camera import FisheyeCamera
    from packnet_sfm_amd.geometry.pose import Pose
    z = gu.load_golden("fisheye_small")
    B, _, H, W = z["depth"].shape
    cam = FisheyeCamera(_intr(z), image_size=(H, W))
    X = cam.reconstruct(_T(z["depth"]), frame="c")
    assert gu.rel_err(X, z["points"]) < 1e-6
    assert gu.rel_err(cam.reconstruct(_T(z["depth"]), frame="w"), z["points"]) < 1e-6   # identity pose
    ref_cam = FisheyeCamera(_intr(z), Tcw=Pose.from_vec(_T(z["vec"]), "euler"), image_size=(H, W))
    assert gu.rel_err(ref_cam.project(X, frame="w"), z["coords"]) < 1e-5
    flat = ref_cam.project(X.view(B, 3, -1), frame="w")           # [B,3,N] point cloud form
    assert gu.rel_err(flat.view(B, H, W, 2), z["coords"]) < 1e-5


def test_scaled_matches_loss_intrinsics():
    from packnet_sfm_amd.geometry.camera import FisheyeCamera
    from oracle import photometric_oracle as O
    z = gu.load_golden("fisheye_small")
    cam = FisheyeCamera(_intr(z), image_size=(24, 80)).scaled(0.5)
    ref = O.fisheye_scale(_intr(z), 0.5, 0.5)
    assert torch.equal(cam.ux, ref["ux"]) and torch.equal(cam.uy, ref["uy"]) and torch.equal(cam.s, ref["s"])
    assert cam.image_size == (12, 40)
