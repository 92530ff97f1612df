"""SfmModel (packnet_sfm/models/SfmModel.py:11-127): depth net (+ optional flip, + upsample of all
inverse-depth scales to full resolution) and pose net (vectors -> Pose)."""
import random

import torch

from ..geometry.pose import Pose
from .base_model import BaseModel
from .model_utils import flip_batch_input, flip_output, upsample_output
from ..datasets.synthetic import flatten_cameras
from ..utils.misc import filter_dict


class SfmModel(BaseModel):
    """`overlap_pose_net`: on a ROCm device, run the pose net on a side HIP stream forked from the
    current one (it depends only on the input images), concurrently with the depth net; its
    backward runs on the same side stream.  Captured into the training-step HIP graph as a
    parallel branch.  Numerically identical to the serial order.

    The pose net is enqueued after the depth net: the autograd engine runs ready nodes in
    decreasing creation order, so the pose backward is then enqueued right after the loss
    backward and its branch runs beside the depth backward.  Enqueued first (the reference's
    order), it came last in the engine's order and ran after the depth backward on the GPU too,
    ~100 small kernels alone at the end of every step."""

    def __init__(self, depth_net=None, pose_net=None, rotation_mode="euler", flip_lr_prob=0.0,
                 upsample_depth_maps=False, overlap_pose_net=True, lazy_upsample=True, **kwargs):
        super().__init__()
        # lazy_upsample: the training-mode upsampled 'inv_depths' are NearestScales (the loss reads
        # the depth net's stored maps; models/model_utils.upsample_output)
        self.lazy_upsample = lazy_upsample
        self.overlap_pose_net = overlap_pose_net
        # A/B (bench.py --pose-first): enqueue the pose branch before the depth net.  Measured equal
        # (profiles/r05/posefirst: 1146-1157 vs 1150-1159 img/s): the graph launch enqueues the branches
        # in node order, so the depth net then waits for the pose forward, and the pose backward runs last
        self.pose_first = False
        self._side_streams = {}
        self.depth_net = depth_net
        self.pose_net = pose_net
        self.rotation_mode = rotation_mode
        self.flip_lr_prob = flip_lr_prob
        self.upsample_depth_maps = upsample_depth_maps
        self._network_requirements = ["depth_net", "pose_net"]

    def add_depth_net(self, depth_net):
        self.depth_net = depth_net

    def add_pose_net(self, pose_net):
        self.pose_net = pose_net

    def depth_net_flipping(self, batch, flip, **kwargs):
        inputs = {key: batch[key] for key in filter_dict(batch, self._input_keys)}
        if flip:
            return flip_output(self.depth_net(**flip_batch_input(inputs), **kwargs))
        return self.depth_net(**inputs, **kwargs)

    def compute_depth_net(self, batch, force_flip=False, **kwargs):
        flag = random.random() < self.flip_lr_prob if self.training else force_flip
        output = self.depth_net_flipping(batch, flag, **kwargs)
        if self.training and self.upsample_depth_maps:
            output = upsample_output(output, mode="nearest", align_corners=None, lazy=self.lazy_upsample)
        return output

    def compute_pose_net(self, image, contexts):
        pose_vec = self.pose_net(image, contexts).float()  # pose algebra in fp32 (nets may be bf16)
        return Pose.from_vecs(pose_vec, self.rotation_mode)

    def _side_stream(self, device):
        if device not in self._side_streams:
            self._side_streams[device] = torch.cuda.Stream(device=device)
        return self._side_streams[device]

    def forward(self, batch, return_logs=False, force_flip=False, **kwargs):
        if batch["rgb"].dim() == 5:   # multi-camera samples [B, cams, 3, H, W] (DDAD): cameras -> batch
            batch = flatten_cameras(batch)   # == model_utils.stack_batch for B = 1 (model_utils.py:68-94)
        poses = None
        want_pose = "rgb_context" in batch and self.pose_net is not None
        if want_pose and self.overlap_pose_net and batch["rgb"].is_cuda:
            cur = torch.cuda.current_stream(batch["rgb"].device)
            side = self._side_stream(batch["rgb"].device)
            side.wait_stream(cur)
            if self.pose_first:
                with torch.cuda.stream(side):
                    poses = self.compute_pose_net(batch["rgb"], batch["rgb_context"])
            depth_output = self.compute_depth_net(batch, force_flip=force_flip, **kwargs)
            if not self.pose_first:
                with torch.cuda.stream(side):
                    poses = self.compute_pose_net(batch["rgb"], batch["rgb_context"])
            cur.wait_stream(side)
            for p in poses:  # allocated on the side stream, consumed on the current one
                p.mat.record_stream(cur)
        else:
            depth_output = self.compute_depth_net(batch, force_flip=force_flip, **kwargs)
            if want_pose:
                poses = self.compute_pose_net(batch["rgb"], batch["rgb_context"])
        return {**depth_output, "poses": poses}
