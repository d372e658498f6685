"""lib.layers — Soft_NN feature matcher and Sampler (reference lib/layers.py)
on MI355X.

Soft_NN.forward keeps the reference contract (x_f [b,n,c], y_f [b,m,c],
y_c [b,m,3] -> x_corr [b,n,3]) but never materialises the [b,n,m] distance
or softmax matrices: one fused HIP kernel (mvr_feat_nn) per call.
Sampler draws its indices with the host numpy RNG exactly as the reference
(np.random.choice, lib/layers.py:145-148) so seeded runs select the same
points, then gathers rows on the device (mvr_gather_rows); 'fps' runs the
furthest-point-sampling kernel (mvr_fps).
"""
import numpy as np
import torch

from lib import _native as N


class Soft_NN(torch.nn.Module):
    """lib/layers.py:10-88.  corr_type in {'soft', 'hard', 'soft_gumbel'}; st = straight-through."""

    def __init__(self, corr_type="soft", st=True, temp=0.3, min_temp=1e-4, device="cuda"):
        super().__init__()
        assert corr_type in ["soft", "hard", "soft_gumbel"], \
            "Wrong correspondence type selected. Must be one of [soft, soft_gumbel, hard]"
        if corr_type == "hard":
            print("Gradients cannot be backpropagated to the feature descriptor because hard NN search is selected.")
        self.device = device
        self.corr_type = corr_type
        self.st = st
        self.min_temp_value = float(min_temp)
        self.register_buffer("min_temp", torch.tensor([min_temp]), persistent=False)
        self._temperature = torch.nn.Parameter(torch.tensor(temp, dtype=torch.float32))
        self._tcache = (None, None)

    def get_temp(self):
        return torch.max(self._temperature ** 2, self.min_temp.to(self._temperature))

    def _inv_tau2(self):
        ver = (self._temperature.data_ptr(), self._temperature._version)
        if self._tcache[0] != ver:
            t = float(self._temperature.detach().float().cpu())
            self._tcache = (ver, 1.0 / max(np.float32(t) * np.float32(t), np.float32(self.min_temp_value)))
        return self._tcache[1]

    def mode(self):
        if self.corr_type == "soft":
            return 1 if self.st else 0
        if self.corr_type == "hard":
            return 1
        return 3 if self.st else 2   # soft_gumbel: hard (straight-through forward value) / soft

    def _gumbel_seed(self):
        """soft_gumbel's noise seed: one draw from torch's default (CPU) generator per call, so torch.manual_seed
        makes runs repeatable as in the reference (whose noise comes from F.gumbel_softmax's own draws)"""
        return int(torch.randint(0, 2 ** 62, (1,), dtype=torch.int64).item())

    def _gumbel(self, Fq, fq_fs, Ft, ft_fs, Xq, xq_fs, Xt, xt_fs, pairs, P, n, m, out, o_ps, o_ns):
        """lib/layers.py:72-78 (F.gumbel_softmax(-dist, tau=get_temp(), hard=st)) on the feature-NN kernel's online
        path with counter-based noise (csrc/feat_nn.hip nn_gumbel_z; oracle/soft_nn.py restates it)"""
        N.check(N.lib().mvr_feat_nn_gumbel(Fq, fq_fs, Ft, ft_fs, Xq, xq_fs, Xt, xt_fs, N.ptr(pairs), P, n, m, 32,
                                           self._inv_tau2(), int(self.st), self._gumbel_seed(), N.ptr(out), o_ps,
                                           o_ns, None, N.stream()), "mvr_feat_nn_gumbel")
        return out

    def match_pairs(self, f_frag, xyz_frag, pairs, out, out_pstride, out_nstride, with_query_xyz=True):
        """Fused pairwise matching over fragments: f_frag [B,n,32], xyz_frag [B,n,3],
        pairs int64 [P,2] (query frag, target frag) -> out(p, i, :) = [xyz_q | x_corr]."""
        P = pairs.shape[0]
        B, n, C = f_frag.shape
        if self.corr_type == "soft_gumbel":
            return self._gumbel(N.ptr(f_frag), n * C, N.ptr(f_frag), n * C, N.ptr(xyz_frag) if with_query_xyz else None,
                                n * 3, N.ptr(xyz_frag), n * 3, pairs, P, n, n, out, out_pstride, out_nstride)
        L = N.lib()
        ws = N.workspace(L.mvr_feat_nn_workspace_bytes(B, n), f_frag.device)   # pre-split target stages
        N.check(L.mvr_feat_nn_ws(N.ptr(f_frag), n * C, N.ptr(f_frag), n * C,
                                 N.ptr(xyz_frag) if with_query_xyz else None, n * 3, N.ptr(xyz_frag), n * 3,
                                 N.ptr(pairs), P, n, n, C, self._inv_tau2(), self.mode(), N.ptr(out),
                                 out_pstride, out_nstride, None, B, N.ptr(ws), ws.numel(), N.stream()), "mvr_feat_nn_ws")
        return out

    def forward(self, x_f, y_f, y_c):
        N.require_hip(x_f)
        b, n, c = x_f.shape
        m = y_f.shape[1]
        if c != 32:
            raise ValueError("the fused matcher expects 32-dim FCGF descriptors")
        x_f = x_f.float().contiguous()
        y_f = y_f.float().contiguous()
        y_c = y_c.float().contiguous()
        pairs = torch.arange(b, device=x_f.device, dtype=torch.int64).repeat_interleave(2).view(b, 2)
        out = torch.empty(b, n, 3, device=x_f.device, dtype=torch.float32)
        if self.corr_type == "soft_gumbel":
            return self._gumbel(N.ptr(x_f), n * c, N.ptr(y_f), m * c, None, 0, N.ptr(y_c), m * 3, pairs, b, n, m, out,
                                n * 3, 3)
        N.check(N.lib().mvr_feat_nn(N.ptr(x_f), n * c, N.ptr(y_f), m * c, None, 0, N.ptr(y_c), m * 3, N.ptr(pairs),
                                    b, n, m, c, self._inv_tau2(), self.mode(), N.ptr(out), n * 3, 3, None,
                                    N.stream()), "mvr_feat_nn")
        return out


class Sampler(torch.nn.Module):
    """lib/layers.py:90-154.  samp_type in {'fps', 'rand'}."""

    def __init__(self, samp_type="fps", targeted_num_points=2000):
        super().__init__()
        assert samp_type in ["fps", "rand"], "Wrong sampling type selected. Must be one of [fps, rand]"
        self.samp_type = samp_type
        self.targeted_num_points = targeted_num_points

    @staticmethod
    def _pts(pts_list):
        return tuple(int(p) for p in (pts_list.cpu().numpy() if torch.is_tensor(pts_list) else pts_list))

    def _rand_indices(self, pts):
        """The reference's draws (lib/layers.py:128-148): one np.random.choice per fragment, in order, on
        numpy's global RandomState.  Without replacement (every fragment has >= targeted points) the
        library replays numpy's own shuffle draw for draw (mvr_sample_rand_mt19937: ~10x numpy's loop)
        and hands the advanced MT19937 state back to numpy."""
        tgt = self.targeted_num_points
        num_points = min(tgt, min(pts))
        st = np.random.get_state()
        if num_points >= tgt and st[0] == "MT19937":
            key = np.array(st[1], dtype=np.uint32, copy=True)
            pos = np.array([st[2]], dtype=np.int32)
            counts = np.asarray(pts, dtype=np.int64)
            out = np.empty((len(pts), tgt), dtype=np.int64)
            ws = np.empty(max(max(pts), 1), dtype=np.int64)
            N.check(N.lib().mvr_sample_rand_mt19937(key.ctypes.data, pos.ctypes.data, counts.ctypes.data, len(pts),
                                                    tgt, out.ctypes.data, ws.ctypes.data), "mvr_sample_rand_mt19937")
            np.random.set_state((st[0], key, int(pos[0]), st[3], st[4]))
            return torch.from_numpy(out)
        out, start = [], 0
        for n in pts:
            rng = np.arange(start, start + n)
            out.append(np.random.choice(rng, tgt, replace=not (num_points >= tgt)))
            start += n
        return torch.from_numpy(np.stack(out).astype(np.int64))

    def indices(self, pts_list, input_C=None, k=None):
        """Global row indices [B, targeted] (int64, on the device of input_C for 'fps').  `k` ('fps' only) overrides
        the sample count min(targeted, min(pts_list)): a rank holding some of a scene's fragments passes the
        scene-wide count, so every fragment is sampled as on one GPU."""
        pts = self._pts(pts_list)
        if self.samp_type == "rand":
            return self._rand_indices(pts)
        from lib.fps import furthest_point_sample
        return furthest_point_sample(input_C, pts, min(self.targeted_num_points, min(pts)) if k is None else int(k))

    def forward(self, input_C, input_F, pts_list):
        N.require_hip(input_F)
        return self.gather(input_C, input_F, self.indices(pts_list, input_C))

    def gather(self, input_C, input_F, idx):
        """sampled (coordinates [B, k, 3], features [B, k, C]) at global row indices idx [B, k] (lib/layers.py:
        146-152's index_select per fragment, one launch each for all fragments)"""
        N.require_hip(input_F)
        B = idx.shape[0]
        if idx.device.type == "cpu":
            # the host draws reach the device through pinned memory without blocking the host (a pageable
            # copy would wait for everything already queued on the stream, i.e. the whole FCGF pass)
            idx = idx.pin_memory().to(input_F.device, non_blocking=True)
        idx = idx.reshape(-1).contiguous()
        C = input_F.float().contiguous()
        X = input_C.float().contiguous()
        k = idx.numel() // B
        sf = torch.empty(B, k, C.shape[1], device=C.device)
        sc = torch.empty(B, k, 3, device=C.device)
        L = N.lib()
        N.check(L.mvr_gather_rows(N.ptr(C), C.shape[1], N.ptr(idx), idx.numel(), N.ptr(sf), N.stream()),
                "mvr_gather_rows")
        N.check(L.mvr_gather_rows(N.ptr(X), 3, N.ptr(idx), idx.numel(), N.ptr(sc), N.stream()), "mvr_gather_rows")
        return sc, sf
