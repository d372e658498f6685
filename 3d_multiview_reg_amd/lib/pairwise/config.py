"""Model factories (reference lib/pairwise/config.py:7-80)."""
import torch

from lib.descriptor import descriptor_dict
from lib.filtering import filtering_dict


def get_model(cfg, device):
    from lib import pairwise
    filtering_module = get_filter(cfg, device)
    descriptor_module = get_descriptor(cfg, device)
    return pairwise.PairwiseReg(descriptor_module=descriptor_module, filtering_module=filtering_module,
                                device=device, samp_type=cfg["train"]["samp_type"],
                                corr_type=cfg["train"]["corr_type"], connectivity_info=None,
                                tgt_num_points=cfg["data"]["max_num_points"],
                                straight_through_gradient=cfg["train"]["st_grad_flag"]).to(device)


def get_descriptor(cfg, device):
    name = cfg["method"]["descriptor_module"]
    if not name:
        return None
    return descriptor_dict[name]().to(device)


def get_filter(cfg, device):
    name = cfg["method"]["filter_module"]
    if not name:
        return None
    return filtering_dict[name](cfg).to(device)


def get_trainer(cfg, model, optimizer, logger, device):
    raise NotImplementedError("training (lib/pairwise/training.py) is outside the MI355X inference hot path")
