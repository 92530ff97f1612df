"""SfmModel (packnet_sfm/models/SfmModel.py:11-127): depth net (+ optional flip, + upsample of all
inverse-depth scales to full resolution) and pose net (vectors -> Pose)."""
import random

from ..geometry.pose import Pose
from .base_model import BaseModel
from .model_utils import flip_batch_input, flip_output, upsample_output
from ..utils.misc import filter_dict


class SfmModel(BaseModel):
    def __init__(self, depth_net=None, pose_net=None, rotation_mode="euler", flip_lr_prob=0.0,
                 upsample_depth_maps=False, **kwargs):
        super().__init__()
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
            output = upsample_output(output, mode="nearest", align_corners=None)
        return output

    def compute_pose_net(self, image, contexts):
        pose_vec = self.pose_net(image, contexts).float()  # pose algebra in fp32 (nets may be bf16)
        return [Pose.from_vec(pose_vec[:, i], self.rotation_mode) for i in range(pose_vec.shape[1])]

    def forward(self, batch, return_logs=False, force_flip=False, **kwargs):
        depth_output = self.compute_depth_net(batch, force_flip=force_flip, **kwargs)
        poses = None
        if "rgb_context" in batch and self.pose_net is not None:
            poses = self.compute_pose_net(batch["rgb"], batch["rgb_context"])
        return {**depth_output, "poses": poses}
