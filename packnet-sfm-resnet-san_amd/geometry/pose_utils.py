"""Pose algebra (host-side torch, differentiable; [B,6] -> [B,4,4] is negligible work).

Mirrors packnet_sfm/geometry/pose_utils.py: `euler2mat` (:8-37), `pose_vec2mat` (:41-51),
`invert_pose` (:55-60), `invert_pose_numpy` (:64-69).
"""
import numpy as np
import torch


def _rot(c, s, axis):
    """Elementary rotation matrices [B,3,3] about x / y / z."""
    o = torch.zeros_like(c)
    l = torch.ones_like(c)
    rows = {
        "x": [l, o, o, o, c, -s, o, s, c],
        "y": [c, o, s, o, l, o, -s, o, c],
        "z": [c, -s, o, s, c, o, o, o, l],
    }[axis]
    return torch.stack(rows, dim=1).view(-1, 3, 3)


def euler2mat(angle):
    """R = Rx(angle[:,0]) @ Ry(angle[:,1]) @ Rz(angle[:,2]) for a [B,3] batch of angles."""
    x, y, z = angle[:, 0], angle[:, 1], angle[:, 2]
    return _rot(x.cos(), x.sin(), "x").bmm(_rot(y.cos(), y.sin(), "y")).bmm(_rot(z.cos(), z.sin(), "z"))


def pose_vec2mat(vec, mode="euler"):
    """[B,6] (tx,ty,tz,rx,ry,rz) -> [B,3,4] = [R|t]."""
    if mode is None:
        return vec
    if mode != "euler":
        raise ValueError("Rotation mode not supported {}".format(mode))
    return torch.cat([euler2mat(vec[:, 3:]), vec[:, :3].unsqueeze(-1)], dim=2)


def invert_pose(T):
    """Inverse of a batch of rigid transforms [B,4,4]: [R^T | -R^T t]."""
    Rt = T[:, :3, :3].transpose(-2, -1)
    t = -Rt.bmm(T[:, :3, 3:])
    bottom = torch.zeros_like(T[:, 3:, :])
    bottom[:, :, 3] = 1.0
    return torch.cat([torch.cat([Rt, t], 2), bottom], 1)


def invert_pose_numpy(T):
    """Inverse of a single [4,4] numpy transform."""
    out = np.eye(4, dtype=T.dtype)
    out[:3, :3] = T[:3, :3].T
    out[:3, 3] = -T[:3, :3].T @ T[:3, 3]
    return out
