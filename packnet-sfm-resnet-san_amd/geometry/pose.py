"""Pose: a batch of [B,4,4] rigid transforms.  Same API as packnet_sfm/geometry/pose.py:8-101
(`identity`, `from_vec`, `inverse`, `transform_pose`, `transform_points`, `@`)."""
import torch

from ._hip_pose import pose_mats_from_vecs
from .pose_utils import invert_pose, pose_vec2mat


class Pose:
    def __init__(self, mat):
        assert tuple(mat.shape[-2:]) == (4, 4)
        self.mat = mat.unsqueeze(0) if mat.dim() == 2 else mat
        assert self.mat.dim() == 3

    def __len__(self):
        return len(self.mat)

    @classmethod
    def identity(cls, N=1, device=None, dtype=torch.float):
        return cls(torch.eye(4, device=device, dtype=dtype).repeat([N, 1, 1]))

    @classmethod
    def from_vec(cls, vec, mode):
        """[B,6] vector -> Pose (pose.py:39-46).  Device fp32 vectors, mode 'euler': one HIP
        launch each way (geometry/_hip_pose.py)."""
        if mode == "euler" and vec.is_cuda and vec.dtype == torch.float32:
            return cls(pose_mats_from_vecs(vec.reshape(len(vec), 1, 6))[0])
        top = pose_vec2mat(vec, mode)
        bottom = torch.zeros(len(vec), 1, 4, device=vec.device, dtype=vec.dtype)
        bottom[:, 0, 3] = 1.0
        return cls(torch.cat([top, bottom], 1))

    @classmethod
    def from_vecs(cls, vec, mode):
        """[B,N,6] (a pose net's output) -> N Poses, [Pose.from_vec(vec[:, i], mode) for i]; on the
        device one launch for all contexts."""
        if mode == "euler" and vec.is_cuda and vec.dtype == torch.float32:
            return [cls(m) for m in pose_mats_from_vecs(vec)]
        return [cls.from_vec(vec[:, i], mode) for i in range(vec.shape[1])]

    @property
    def shape(self):
        return self.mat.shape

    def item(self):
        return self.mat

    def repeat(self, *args, **kwargs):
        self.mat = self.mat.repeat(*args, **kwargs)
        return self

    def inverse(self):
        return Pose(invert_pose(self.mat))

    def to(self, *args, **kwargs):
        self.mat = self.mat.to(*args, **kwargs)
        return self

    def transform_pose(self, pose):
        assert tuple(pose.shape[-2:]) == (4, 4)
        return Pose(self.mat.bmm(pose.item()))

    def transform_points(self, points):
        """R X + t for points [B,3,H,W] (or [B,3,N])."""
        assert points.shape[1] == 3
        B = points.shape[0]
        flat = points.reshape(B, 3, -1)
        out = self.mat[:, :3, :3].bmm(flat) + self.mat[:, :3, 3:]
        return out.view(points.shape)

    def __matmul__(self, other):
        if isinstance(other, Pose):
            return self.transform_pose(other)
        if isinstance(other, torch.Tensor):
            if other.shape[1] == 3 and other.dim() in (3, 4):
                return self.transform_points(other)
            raise ValueError("Unknown tensor dimensions {}".format(other.shape))
        raise NotImplementedError()
