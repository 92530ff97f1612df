"""packnet_sfm_amd — MI355X-native self-supervised depth training step.

Mirrors the reference's `packnet_sfm` call surface for the photometric hot path
(SfmModel / SelfSupModel / MultiViewPhotometricLoss / Camera / Pose / view_synthesis);
the view-synthesis + SSIM/L1 + min-reprojection + smoothness inner loop runs as
hand-written HIP kernels for gfx950 (csrc/, C-ABI in include/psfm.h).
"""
__version__ = "0.1.0"
