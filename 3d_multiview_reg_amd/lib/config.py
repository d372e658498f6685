"""Method registry and model factory (reference lib/config.py:5-47)."""
import torch

from lib import pairwise

method_dict = {
    'pairwise': pairwise,
}


def get_model(cfg):
    method = cfg['method']['task']
    device = torch.device('cuda' if (torch.cuda.is_available() and cfg['misc']['use_gpu']) else 'cpu')
    return method_dict[method].config.get_model(cfg, device=device)


def get_trainer(cfg, model, optimizer, logger):
    method = cfg['method']['task']
    device = torch.device('cuda' if (torch.cuda.is_available() and cfg['misc']['use_gpu']) else 'cpu')
    return method_dict[method].config.get_trainer(cfg, model, optimizer, logger, device)
