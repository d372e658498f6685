"""Checkpoint I/O (reference lib/checkpoints.py:13-133), same API and
state-dict layout ({'model': PairwiseReg.state_dict(), scalars...}).
Files are read with torch.load(weights_only=True): tensors and plain scalars only."""
import os
import urllib.parse

import torch


def is_url(url):
    return urllib.parse.urlparse(url).scheme in ("http", "https")


class CheckpointIO(object):
    def __init__(self, checkpoint_dir="./chkpts", initialize_from=None, initialization_file_name="model_best.pt",
                 **kwargs):
        self.module_dict = kwargs
        self.checkpoint_dir = checkpoint_dir
        self.initialize_from = initialize_from
        self.initialization_file_name = initialization_file_name
        if checkpoint_dir != "" and not os.path.exists(checkpoint_dir):
            os.makedirs(checkpoint_dir)

    def register_modules(self, **kwargs):
        self.module_dict.update(kwargs)

    def save(self, filename, **kwargs):
        if not os.path.isabs(filename):
            filename = os.path.join(self.checkpoint_dir, filename)
        out = dict(kwargs)
        for k, v in self.module_dict.items():
            out[k] = v.state_dict()
        torch.save(out, filename)

    def load(self, filename="model.pt"):
        if is_url(filename):
            raise RuntimeError("checkpoint URLs are not fetched (offline); stage the file locally")
        return self.load_file(filename)

    def load_file(self, filename):
        if not os.path.isabs(filename):
            filename = os.path.join(self.checkpoint_dir, filename)
        if os.path.exists(filename):
            print(filename)
            print("=> Loading checkpoint from local file...")
            return self.parse_state_dict(torch.load(filename, map_location="cpu", weights_only=True))
        if self.initialize_from is not None:
            path = os.path.join(self.initialize_from, self.initialization_file_name)
            if os.path.exists(path):
                return self.parse_state_dict(torch.load(path, map_location="cpu", weights_only=True))
        raise FileExistsError(filename)

    def parse_state_dict(self, state_dict):
        for k, v in self.module_dict.items():
            if k in state_dict:
                v.load_state_dict(state_dict[k])
            else:
                print("Warning: Could not find %s in checkpoint!" % k)
        return {k: v for k, v in state_dict.items() if k not in self.module_dict}
