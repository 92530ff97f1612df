"""Checkpoint loading (packnet_sfm/utils/load.py:114-163 `load_network`).

A reference checkpoint (models/model_checkpoint.py:66-76) holds ModelWrapper.state_dict() under
'state_dict', i.e. keys 'model.depth_net.…' / 'model.pose_net.…'.  `load_network(net, ckpt,
'depth_net')` keeps the keys that contain 'depth_net.', strips everything up to and including
that prefix, and loads the entries whose name and shape match the network (strict=False), as the
reference does.  Files are read with torch.load(weights_only=True): nothing in the file executes.
"""
from collections import OrderedDict

import torch


def load_network(network, path, prefixes=""):
    """Load the matching entries of a checkpoint (path or state dict) into `network`; returns
    (network, number of tensors loaded, number of tensors in the network)."""
    prefixes = [prefixes] if isinstance(prefixes, str) else list(prefixes)
    if isinstance(path, str):
        saved = torch.load(path, map_location="cpu", weights_only=True)["state_dict"]
    else:
        saved = path
    own = network.state_dict()
    updated, n = OrderedDict(), 0
    for key, val in saved.items():
        for prefix in prefixes:
            prefix = prefix + "."
            if prefix in key:
                k = key[key.find(prefix) + len(prefix):]
                if k in own and tuple(val.shape) == tuple(own[k].shape):
                    updated[k] = val
                    n += 1
    network.load_state_dict(updated, strict=False)
    return network, n, len(own)
