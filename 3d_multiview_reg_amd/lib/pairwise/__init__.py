"""PairwiseReg (reference lib/pairwise/__init__.py:15-142) on MI355X.

compute_descriptors runs the whole front of the hot path on the device with
no [P, n, *] pair tensors and no [P, n, n] distance matrices:
  FCGF (batched over all fragments) -> Sampler (host np.random indices, device
  gather) -> fused feature-NN over the C(B,2) pair list (lib.utils.pair_index
  order) writing the OANet input xs [P, n, 6] directly.
The reverse matching (t -> s) the reference computes at
lib/pairwise/__init__.py:111 is skipped: its result only feeds the mutual
side channel, which the reference never passes on (its call at :120 shifts the
argument) — outputs are identical.
"""
import torch
import torch.nn as nn

from lib.layers import Soft_NN, Sampler
from lib.sparse import SparseTensor
from lib.utils import pair_index, construct_filtering_input_data, extract_mutuals
from lib.pairwise import config  # noqa: F401

__all__ = ["PairwiseReg", "config"]


class PairwiseReg(nn.Module):
    def __init__(self, descriptor_module, filtering_module, device, samp_type="fps", corr_type="soft",
                 mutuals_flag=False, connectivity_info=None, tgt_num_points=2000, straight_through_gradient=True,
                 train_descriptor=False):
        super().__init__()
        self.device = device
        self.samp_type = samp_type
        self.corr_type = corr_type
        self.mutuals = mutuals_flag
        self.connectivity_info = connectivity_info
        self.train_descriptor = train_descriptor
        self.descriptor_module = descriptor_module
        if self.descriptor_module:
            self.sampler = Sampler(samp_type=self.samp_type, targeted_num_points=tgt_num_points)
            self.feature_matching = Soft_NN(corr_type=self.corr_type, st=straight_through_gradient)
            self.precomputed_desc = False
        else:
            self.precomputed_desc = True
        self.filtering_module = filtering_module

    def forward(self, data):
        filtering_input, f_0, f_1 = self.compute_descriptors(input_dict=data)
        registration_outputs = self.filter_correspondences(filtering_input)
        return filtering_input, f_0, f_1, registration_outputs

    def compute_descriptors(self, input_dict):
        if self.precomputed_desc:
            return input_dict, None, None
        return self.match_samples(input_dict, *self.sample_descriptors(input_dict))

    def sample_descriptors(self, input_dict):
        """First stage of compute_descriptors: FCGF + Sampler -> (xyz_b [B,n,3], f_b [B,n,32], F0, F1)."""
        dev = next(self.descriptor_module.parameters()).device
        xyz_down = input_dict["pcd0"].to(dev).float().contiguous()
        pts_list = input_dict["pts_list"]
        if input_dict.get("sinput0_coords_manager") is not None:
            # a prepared lib.sparse.CoordinateManager of sinput0_C (its strided coordinate sets already built,
            # e.g. one scene ahead on another stream): the FCGF launches then need no host synchronisation
            sinput0 = SparseTensor(input_dict["sinput0_F"], coords_manager=input_dict["sinput0_coords_manager"]).to(dev)
        else:
            sinput0 = SparseTensor(input_dict["sinput0_F"], coords=input_dict["sinput0_C"],
                                   batch_size=len(pts_list)).to(dev)
        F0 = self.descriptor_module(sinput0).F
        if self.train_descriptor:
            sinput1 = SparseTensor(input_dict["sinput1_F"], coords=input_dict["sinput1_C"]).to(dev)
            F1 = self.descriptor_module(sinput1).F
        else:
            F1 = torch.empty(F0.shape[0], 0, device=dev)
        xyz_b, f_b = self.sampler(xyz_down, F0, pts_list)                      # [B, n, 3], [B, n, 32]
        return xyz_b, f_b, F0, F1

    def match_samples(self, input_dict, xyz_b, f_b, F0, F1):
        """Second stage of compute_descriptors: feature NN over the pair list -> filtering input."""
        dev = xyz_b.device
        B, n = xyz_b.shape[0], xyz_b.shape[1]
        if self.connectivity_info is not None:
            pairs = torch.as_tensor(self.connectivity_info, dtype=torch.int64, device=dev).reshape(-1, 2)
        else:
            pairs = pair_index(B, dev)
        pairs = pairs.contiguous()
        P = pairs.shape[0]
        xs = torch.empty(P, n, 6, device=dev)
        self.feature_matching.match_pairs(f_b, xyz_b, pairs, xs, n * 6, 6)      # [x_s | NN_s->t]
        if self.mutuals:
            # computed like the reference (lib/pairwise/__init__.py:110-117) but, as there, not fed to the filter
            back = torch.empty(P, n, 3, device=dev)
            self.feature_matching.match_pairs(f_b, xyz_b, pairs.flip(1).contiguous(), back, n * 3, 3,
                                              with_query_xyz=False)
            extract_mutuals(xs[..., :3], xyz_b[pairs[:, 1]], xs[..., 3:], back)
        if "T_global_0" in input_dict:   # GT residuals / labels (lib/utils.py:906-908)
            filtering_input = construct_filtering_input_data(xs[..., :3], xs[..., 3:], input_dict, pairs)
        else:                            # lib/utils.py:910-913: host-side placeholders, as the reference
            filtering_input = {"ys": torch.zeros(P, n, 1), "Rs": torch.eye(3).unsqueeze(0).repeat(P, 1, 1),
                               "ts": torch.zeros(P, 3, 1)}
        filtering_input["xs"] = xs.unsqueeze(1)                                   # the fused buffer, [P,1,n,6]
        return filtering_input, F0, F1

    def filter_correspondences(self, input_dict):
        return self.filtering_module(input_dict)
