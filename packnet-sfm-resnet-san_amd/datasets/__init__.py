"""GPU mirror of packnet_sfm/datasets transforms."""
from .augmentations import (augment_images, random_color_jitter_params, train_transforms_batch,  # noqa: F401
                            validation_transforms_batch)
from .transforms import get_transforms, train_transforms, validation_transforms  # noqa: F401
