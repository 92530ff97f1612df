"""Import shim: the package lives in `packnet-sfm-resnet-san_amd/` (a directory name that is
not a Python identifier).  `import packnet_sfm_amd` loads that directory as the package
`packnet_sfm_amd`, so `from packnet_sfm_amd.losses.multiview_photometric_loss import
MultiViewPhotometricLoss` mirrors the reference's `packnet_sfm.…` import paths."""
import importlib.util
import os
import sys

_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "packnet-sfm-resnet-san_amd")
_spec = importlib.util.spec_from_file_location(
    __name__, os.path.join(_DIR, "__init__.py"), submodule_search_locations=[_DIR])
_mod = importlib.util.module_from_spec(_spec)
sys.modules[__name__] = _mod
_spec.loader.exec_module(_mod)
