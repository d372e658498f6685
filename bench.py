#!/usr/bin/env python3
"""Throughput benchmark of the MI355X pairwise-registration hot path.

  python bench.py [--gpus N] [--steps K] [--warmup W] [--workload scene|precomputed]

One process per GPU (torchrun for N>1, RCCL over xGMI).  A *step* is one pass
of the hot path over one batch of synthetic input resident in HBM:

  scene        (default, BASELINE configs[2]: one 3DMatch-scale scene per GPU)
               30 fragments of ~20k voxels -> FCGF descriptors -> rand sampling
               (5000 pts) -> feature NN for all 435 pairs -> OANet -> Procrustes
               -> RCCL all-gather of the per-pair (R, t, conf) records.
  precomputed  (BASELINE configs[3] shape: the benchmark's precomputed
               correspondences) 435 pairs x 5000 correspondences -> OANet ->
               Procrustes -> all-gather.

Weak scaling: every rank processes its own scene / pair batch (different seed).
Rank 0 prints ONE JSON line (the driver contract); the roofline object prices
the dominant kernel class from per-launch hipEvent timings taken inside the
timed region (plus the SURVEY §8d whole-step floor); cpu_baseline times the
reference's CPU op sequence (oracle/torch_port.py, numpy FCGF restatement) on a
bounded sample of the same workload on this host's cores, and on 8 threads.
"""
import argparse
import json
import os
import sys
import time
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.abspath(__file__))
for p in (os.path.join(ROOT, "3d_multiview_reg_amd"), ROOT, os.path.join(ROOT, "tests", "golden")):
    if p not in sys.path:
        sys.path.insert(0, p)

import numpy as np  # noqa: E402
import torch  # noqa: E402

METRIC = "point-cloud pairs/s (feat+match+filter+SVD), 3DMatch 20k-pt, 1/2/4/8 GPU"
PEAK_FP32_TFLOPS = 157.3    # MI355X dense fp32 (vector == MFMA), MI355X_MICROARCH.md
PEAK_BF16_TFLOPS = 16 * PEAK_FP32_TFLOPS   # dense bf16 MFMA (fp32 MFMA is 1/16 of it)
# the OANet GEMMs run the 3-term bf16 split (6 bf16 MFMA products per fp32 product, csrc/gemm.hpp):
# their fp32-equivalent MFMA ceiling
PEAK_SPLIT_TFLOPS = PEAK_BF16_TFLOPS / 6
PEAK_HBM_GBS = 8000.0
GEMM_CLASSES = ("conv_pts", "embed", "pool", "unpool", "oafilter")


def log(*a):
    if int(os.environ.get("RANK", "0")) == 0:
        print(*a, file=sys.stderr, flush=True)


def oanet_cfg():
    # configs/pairwise_registration/eval/RegBlock.yaml
    return {"misc": {"net_depth": 12, "clusters": 500, "iter_num": 1, "net_channel": 128, "use_gpu": True,
                     "normalize_weights": True}, "data": {"use_mutuals": 0, "max_num_points": 5000},
            "method": {"task": "pairwise", "descriptor_module": None, "filter_module": "oanet"},
            "train": {"samp_type": "rand", "corr_type": "soft", "st_grad_flag": False}}


def synth_module(mod, seed):
    from synth import synth_state
    shapes = {k: tuple(v.shape) for k, v in mod.state_dict().items()}
    st = synth_state(shapes, seed=seed)
    mod.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    return st


class PrecomputedWorkload:
    """configs[3]/[4] shape: scripts/benchmark_pairwise_registration.py's hot loop (:193-200) on precomputed
    correspondences — loader batches of 32 pairs, each one filter_correspondences call in TRAIN-mode BatchNorm
    (the script never calls model.eval(), :159-174: batch statistics per 32-pair batch, the zero-row guard per
    batch), then Procrustes."""
    name = "precomputed"
    BATCH = 32

    def __init__(self, dev, rank, pairs, npts, shard="scenes", world=1):
        from lib.filtering.oanet import OANet
        from lib import distributed as D
        from synth import synth_correspondences
        self.net = OANet(oanet_cfg())
        self.state = synth_module(self.net, seed=7)
        self.net = self.net.to(dev).train()
        # the loader batches side by side in one forward: BatchNorm statistics and the zero-row guard per 32-pair
        # group, exactly the per-batch semantics (tests/test_gpu_oanet.py::test_oanet_bn_groups_equal_batches);
        # MVR_PRECOMP_SEQUENTIAL=1 runs one forward per batch instead
        self.grouped = os.environ.get("MVR_PRECOMP_SEQUENTIAL", "0") != "1"
        if self.grouped:
            self.net.bn_group = self.BATCH
            self.net.guard_group = self.BATCH
        # scenes: every rank its own evaluation (weak scaling); pairs: ONE evaluation, its loader batches split into
        # contiguous blocks of whole 32-pair batches over the ranks (lib.distributed.shard_pairs, the harness's
        # --dist split: scripts/benchmark_pairwise_registration.py under torchrun), records all-gathered
        self.shard, self.world = shard, world
        xs, _, _ = synth_correspondences(pairs, npts, seed=1000 + (rank if shard == "scenes" else 0))
        self.p0, self.p1 = D.shard_pairs(pairs, world, rank, group=self.BATCH) if shard == "pairs" else (0, pairs)
        xs = np.ascontiguousarray(xs[self.p0:self.p1])
        self.xs_host = xs
        self.xs = torch.from_numpy(xs).to(dev).unsqueeze(1)
        self.pairs = pairs
        self.npts = npts
        self.dev = dev

    def step(self):
        if self.xs.shape[0] == 0:                          # an empty block (more ranks than loader batches)
            return torch.zeros(0, 13, device=self.dev)
        if self.grouped:
            out = self.net({"xs": self.xs})
            R, t, s = out["rot_est"][-1], out["trans_est"][-1], out["scores"][-1]
            conf = (s > 0.5).float().mean(dim=1, keepdim=True)
            return torch.cat([R.reshape(-1, 9), t.reshape(-1, 3), conf], dim=1)
        recs = []
        for b0 in range(0, self.pairs, self.BATCH):
            out = self.net({"xs": self.xs[b0:b0 + self.BATCH]})
            R, t, s = out["rot_est"][-1], out["trans_est"][-1], out["scores"][-1]
            conf = (s > 0.5).float().mean(dim=1, keepdim=True)
            recs.append(torch.cat([R.reshape(-1, 9), t.reshape(-1, 3), conf], dim=1))   # [b, 13] records
        return torch.cat(recs)

    def gather(self, rec, world):
        if self.shard == "pairs":
            from lib import distributed as D
            return D.gather_records(rec, self.pairs, world, group=self.BATCH) if world > 1 else rec
        return records_allgather(rec, world)

    def config(self):
        return {"workload": "precomputed correspondences (configs[3] shape, scripts/benchmark_pairwise_registration.py "
                            "hot loop): OANet(128ch,500 clusters,depth 12,2 blocks, train-mode BN per 32-pair batch)"
                            "+Procrustes" + (": ONE evaluation of %d pairs, its 32-pair batches split over %d ranks"
                                             % (self.pairs, self.world) if self.shard == "pairs" else ""),
                "pairs_per_gpu": self.p1 - self.p0 if self.shard == "pairs" else self.pairs,
                "correspondences": self.npts,
                "batch": self.BATCH, "batches": "one forward, per-batch BN / guard groups" if self.grouped else
                "one forward per batch"}

    def cpu_baseline(self, threads, budget_s=20.0):
        """the reference's op sequence on torch CPU tensors (oracle/torch_port.py: N x N diag_embed Kabsch) over
        whole 32-pair batches of the same workload, train-mode BN"""
        from oracle import torch_port
        torch.set_num_threads(threads)
        n, t0 = 0, time.time()
        with torch.no_grad():
            while n < self.pairs and (n == 0 or time.time() - t0 < budget_s):
                torch_port.oanet_forward(self.state, torch.from_numpy(self.xs_host[n:n + self.BATCH]), train=True)
                n += min(self.BATCH, self.pairs - n)
        dt = time.time() - t0
        return n / dt, ("%d pairs in batches of %d (oracle/torch_port.py, reference op sequence incl. N x N diag_embed "
                        "Kabsch, train-mode BN), measured" % (n, self.BATCH)), \
            {"extrapolated": n < self.pairs, "pairs_timed": n, "batches_timed": -(-n // self.BATCH)}


class SceneWorkload:
    """configs[2]: one synthetic 3DMatch-scale scene per GPU (30 fragments, ~20k voxels each)."""
    name = "scene"

    def __init__(self, dev, rank, npts=5000, n_frag=30, voxel=0.025, samp="rand", shard="scenes", world=1,
                 groups=None, emulate=False):
        import lib.config
        from lib.sparse import fragment_views
        from synth import synth_scene_fragments
        cfg = oanet_cfg()
        cfg["method"]["descriptor_module"] = "fcgf"
        cfg["data"]["max_num_points"] = npts
        cfg["train"]["samp_type"] = samp
        self.samp = samp
        self.model = lib.config.get_model(cfg)
        self.state = synth_module(self.model, seed=7)
        self.model = self.model.to(dev).eval()
        self.shard, self.world, self.rank, self.emulate = shard, world, rank, emulate
        # scenes: every rank its own scene (weak scaling); pairs: ONE scene, its fragments and pairs split over the
        # ranks (strong scaling, north_star's pair-sharded batch)
        self.frags, self.poses = synth_scene_fragments(n_frag, seed=41 + (1000 * rank if shard == "scenes" else 0))
        self.dev, self.voxel, self.npts, self.n_frag = dev, voxel, npts, n_frag
        self.rng_seed = 41 + (rank if shard == "scenes" else 0)
        self.pairs = n_frag * (n_frag - 1) // 2
        self.vox_counts = None
        if shard == "pairs":
            from lib import distributed as D
            from lib.utils import pair_index
            # fragments: contiguous blocks of ceil(n_frag / world) (FCGF + sampling of its block per rank);
            # pairs: contiguous blocks of the lexicographic pair list (feature NN + OANet + Procrustes per rank)
            self.fper = -(-n_frag // world)
            self.f0, self.f1 = min(rank * self.fper, n_frag), min((rank + 1) * self.fper, n_frag)
            self.p0, self.p1 = D.shard_pairs(self.pairs, world, rank, group=1)
            self.pair_block = pair_index(n_frag, dev)[self.p0:self.p1].contiguous()
            self.pg_counts, self.pg_samples, self.pg_filter = groups
            self.raw = fragment_views(self.frags[self.f0:self.f1], dev)
        else:
            self.raw = fragment_views(self.frags, dev)     # resident in HBM, one buffer (voxelize reads it in place)

    def prepare(self):
        """voxelise (prepare_data on the GPU) and build the strided coordinate sets of the sparse input: every
        host synchronisation of the scene (voxel counts, the size of each coordinate level) happens here.
        shard=pairs: this rank's fragments only; the voxel counts of all fragments (the sampler's draws depend on
        them) arrive by one host all-gather (gloo group)."""
        from lib.sparse import voxelize, CoordinateManager
        coords, sel, counts, xyz_down = voxelize(self.raw, self.voxel, self.dev)
        cm = CoordinateManager(coords, len(counts))
        for s in (2, 4, 8):   # FCGF's tensor strides (fcgf.py:118-227)
            cm.coords_at(s)
        d = {"pcd0": xyz_down, "sinput0_C": coords, "sinput0_F": torch.ones(coords.shape[0], 1, device=self.dev),
             "pts_list": torch.tensor(counts), "sinput0_coords_manager": cm}
        if self.shard == "pairs" and self.emulate:   # rank 0 of `world`: every block sized like this rank's
            mine = list(counts) + [counts[-1]] * (self.fper - len(counts))
            d["pts_all"] = counts = (mine * self.world)[:self.n_frag]
        elif self.shard == "pairs":
            import torch.distributed as dist
            mine = torch.full((self.fper,), -1, dtype=torch.int64)
            mine[:len(counts)] = torch.tensor(counts, dtype=torch.int64)
            parts = [torch.empty_like(mine) for _ in range(self.world)]
            dist.all_gather(parts, mine, group=self.pg_counts)
            allc = torch.cat(parts)
            counts = [int(c) for c in allc[allc >= 0]]
            d["pts_all"] = counts
        self.vox_counts = counts
        return d

    def describe(self, data=None):
        """(voxelise ->) FCGF -> Sampler -> feature NN over all pairs (compute_descriptors).
        shard=pairs: FCGF + sampling of this rank's fragments (the sampler's numpy draws replayed for the whole
        scene, lib/layers.py:128-148, so every fragment gets the draws it gets on one GPU), one all-gather of the
        sampled (xyz, descriptor) of every fragment (RCCL, ~21 MB per scene), then the feature NN of this rank's
        block of pairs only."""
        if data is None:
            self._wait_prep()
            data = self.prepare()
        np.random.seed(self.rng_seed)
        if self.shard != "pairs":
            fin, _, _ = self.model.compute_descriptors(data)
            return fin
        from lib import distributed as D
        from lib.sparse import SparseTensor
        m = self.model
        allc = data["pts_all"]
        if self.samp == "rand":
            # the reference's draws always have `targeted` columns (with replacement when a fragment is smaller)
            n = m.sampler.targeted_num_points
            idx = m.sampler.indices(allc)                                 # [n_frag, k] rows of the whole scene
            idx = idx[self.f0:self.f1] - int(np.sum(allc[:self.f0]))      # -> rows of this rank's fragments
        else:                                                             # fps: per fragment, no shared state, but
            n = min(m.sampler.targeted_num_points, min(allc))             # the scene-wide count, as on one GPU
            idx = m.sampler.indices(data["pts_list"], data["pcd0"], k=n) if self.f1 > self.f0 else None
        buf = torch.zeros(self.fper, n, 35, device=self.dev)
        if self.f1 > self.f0:
            F0 = m.descriptor_module(SparseTensor(data["sinput0_F"], coords_manager=data["sinput0_coords_manager"])).F
            sc, sf = m.sampler.gather(data["pcd0"], F0, idx)
            buf[:self.f1 - self.f0, :, :3] = sc
            buf[:self.f1 - self.f0, :, 3:] = sf
        allb = D.all_gather_rows(buf, self.world, self.pg_samples)[:self.n_frag]   # every fragment, pair order
        xyz_b, f_b = allb[..., :3].contiguous(), allb[..., 3:].contiguous()
        xs = torch.empty(self.p1 - self.p0, n, 6, device=self.dev)
        if self.p1 > self.p0:
            m.feature_matching.match_pairs(f_b, xyz_b, self.pair_block, xs, n * 6, 6)
        return {"xs": xs.unsqueeze(1), "num_pairs": self.pairs}

    def finish(self, fin):
        """OANet -> Procrustes -> per-pair records (R, t, inlier fraction).  shard=pairs: this rank's block
        through lib.distributed.register_pairs_sharded (guard over the whole scene's batch, as on one GPU), whose
        RCCL all-gather returns the records of ALL pairs on every rank"""
        if self.shard == "pairs":
            from lib import distributed as D
            rec = D.register_pairs_sharded(self.model, fin, self.world, self.rank, group=1, guard="scene",
                                           pg=self.pg_filter, first_pair=self.p0)
            return rec[:, 1:14]
        out = self.model.filter_correspondences(fin)
        R, t, s = out["rot_est"][-1], out["trans_est"][-1], out["scores"][-1]
        conf = (s > 0.5).float().mean(dim=1, keepdim=True)
        return torch.cat([R.reshape(-1, 9), t.reshape(-1, 3), conf], dim=1)

    def gather(self, rec, world):
        """records of every rank: pairs mode's finish() already returns all pairs"""
        return rec if self.shard == "pairs" else records_allgather(rec, world)

    def step(self):
        return self.finish(self.describe())

    def step_pipelined(self, world):
        """Software pipeline over consecutive scenes on three HIP streams: the filtering (OANet + Procrustes)
        of scene k-1 (stream B, enqueued first) runs while scene k is described by FCGF and matched (stream A),
        and scene k+1 is voxelised with its coordinate levels built (stream C).  Every host synchronisation of
        a scene (voxel counts, level sizes) waits only for stream C's short queue, so the host enqueues the FCGF
        stage without stalls and streams A and B stay fed.  Returns the gathered records of scene k-1 (None on
        the first call)."""
        if not hasattr(self, "streams"):
            # B (OANet, the longer stage) at high priority: its kernels take the CUs first and the FCGF stage
            # fills what they leave free; C (short voxelisation kernels the host waits for) high as well
            self.streams = (torch.cuda.Stream(self.dev), torch.cuda.Stream(self.dev, priority=-1),
                            torch.cuda.Stream(self.dev, priority=-1))
            self.pending = None
            self.prepared = None
        sA, sB, sC = self.streams
        if not hasattr(self, "prep_pool"):
            # the next scene's voxelisation runs in a helper thread: its host synchronisations (voxel counts, level
            # sizes) then never hold up the enqueue of the next step's filtering on stream B
            self.prep_pool = (ThreadPoolExecutor(1) if os.environ.get("MVR_BENCH_PREP_THREAD", "1") == "1" else None)
        rec = None
        if self.pending is not None:
            fin, ev = self.pending
            with torch.cuda.stream(sB):
                sB.wait_event(ev)
                fin["xs"].record_stream(sB)
                rec = self.gather(self.finish(fin), world)
        if self.prepared is None:
            self.prepared = self.prepare_on(sC)
        data, evc = self.prepared.result() if hasattr(self.prepared, "result") else self.prepared
        with torch.cuda.stream(sA):
            sA.wait_event(evc)
            cm = data["sinput0_coords_manager"]
            for t in [data["pcd0"], data["sinput0_C"], data["sinput0_F"]] + list(cm.coords.values()):
                t.record_stream(sA)
            fin = self.describe(data)
            ev = torch.cuda.Event()
            ev.record(sA)
        self.pending = (fin, ev)
        # the next scene (the same synthetic scene, re-voxelised each step)
        self.prepared = self.prep_pool.submit(self.prepare_on, sC) if self.prep_pool else self.prepare_on(sC)
        return rec

    def _wait_prep(self):
        """a prepare() issued from the main thread first waits for the helper thread's pending one: with
        --shard pairs each prepare() makes a collective (the voxel counts), and one rank's two threads must not
        interleave theirs (every rank then issues them in the same order)"""
        p = getattr(self, "prepared", None)
        if p is not None and hasattr(p, "result"):
            p.result()

    def prepare_on(self, stream):
        """prepare() on `stream` (callable from a helper thread: the current device and stream are per thread)"""
        torch.cuda.set_device(self.dev)
        with torch.cuda.stream(stream):
            data = self.prepare()
            ev = torch.cuda.Event()
            ev.record(stream)
        return data, ev

    def config(self):
        if self.shard == "pairs":
            return {"workload": "ONE synthetic 3DMatch-scale scene per step over all ranks (configs[2]/[3] pair "
                                "sharding): %d fragments x ~%d voxels (0.025 m), FCGF + %s %d samples of %d fragments "
                                "per rank -> all-gather of the samples -> soft feature-NN + OANet (128ch, 500 clusters, "
                                "2 blocks) + weighted Procrustes of %d-%d of the %d pairs per rank (scene-wide zero-row "
                                "guard) -> all-gather of (R,t,conf)"
                                % (self.n_frag, int(np.mean(self.vox_counts or [0])), self.samp, self.npts, self.fper,
                                   self.pairs // self.world, -(-self.pairs // self.world), self.pairs),
                    "sampler": self.samp, "fragments": self.n_frag, "pairs": self.pairs,
                    "fragments_per_gpu": self.fper, "pairs_per_gpu": -(-self.pairs // self.world),
                    "samples": self.npts, "voxels_mean": int(np.mean(self.vox_counts or [0]))}
        which = {30: "configs[2]", 50: "configs[4] scene size: a Redwood-scale scene"}.get(self.n_frag, "custom")
        return {"workload": "one synthetic 3DMatch-scale scene per GPU (%s): %d fragments x ~%d voxels "
                            "(0.025 m) -> FCGF -> %s %d samples -> soft feature-NN for all %d pairs -> OANet "
                            "(128ch, 500 clusters, 2 blocks) -> weighted Procrustes -> all-gather of (R,t,conf)"
                            % (which, self.n_frag, int(np.mean(self.vox_counts or [0])), self.samp, self.npts,
                               self.pairs),
                "sampler": self.samp,
                "fragments_per_gpu": self.n_frag, "pairs_per_gpu": self.pairs, "samples": self.npts,
                "voxels_mean": int(np.mean(self.vox_counts or [0]))}

    def cpu_baseline(self, threads, budget_s=20.0):
        """The reference's CPU op sequence, timed on this host's cores: FCGF fragment by fragment in C + OpenMP
        (oracle/csrc/sparse_conv.c behind oracle/fcgf.py: MinkowskiEngine is absent, so this is our sparse-conv
        restatement, "not ME") until every fragment of the scene is done or half the budget is spent, then one
        32-pair batch (the benchmark's batch) through both Soft_NN directions (full [32, 5000, 5000] distance /
        softmax matrices), OANet (eval BN) and the N x N diag_embed Kabsch (oracle/torch_port.py); the scene's
        rate is pairs / (fragments x mean t_fcgf + ceil(pairs / 32) x t_batch): the batches are extrapolated
        from the one timed."""
        from oracle.fcgf import voxelize as ovox, fcgf_forward, set_threads
        from oracle.soft_nn import sample_rand
        from oracle import torch_port
        torch.set_num_threads(threads)
        set_threads(threads)
        st = {k: v.detach().cpu().numpy() for k, v in self.model.state_dict().items()}
        dst = {k[len("descriptor_module."):]: v for k, v in st.items() if k.startswith("descriptor_module.")}
        fst = {k[len("filtering_module."):]: v for k, v in st.items() if k.startswith("filtering_module.")}
        t0 = time.time()
        nf = 0
        for f in self.frags:
            c, sel, cnt = ovox([f], self.voxel)
            F, _ = fcgf_forward(dst, c, np.ones((len(c), 1), np.float32), backend="c")
            if nf == 0:
                F0, sel0, cnt0 = F, sel, cnt
            nf += 1
            if time.time() - t0 > budget_s / 2:
                break
        t_fcgf = (time.time() - t0) / nf
        # one 32-pair batch: the sampled descriptors of one fragment matched against 32 others' (the descriptors'
        # values do not change the op count; the fragment's own are reused)
        xyz = np.ascontiguousarray(self.frags[0][sel0], dtype=np.float32)
        np.random.seed(0)
        idx = sample_rand(cnt0, self.npts)[0]
        B = 32
        fs = torch.from_numpy(np.repeat(F0[idx][None], B, 0))
        ft = torch.from_numpy(np.repeat(F0[np.roll(idx, 17)][None], B, 0))
        xs_, xt_ = torch.from_numpy(np.repeat(xyz[idx][None], B, 0)), torch.from_numpy(np.repeat(xyz[np.roll(idx, 17)][None], B, 0))
        t1 = time.time()
        with torch.no_grad():
            xc = torch_port.soft_nn(fs, ft, xt_)
            torch_port.soft_nn(ft, fs, xs_)                   # the reverse direction, as the reference
            torch_port.oanet_forward(fst, torch.cat([xs_, xc], -1).contiguous())
        t_batch = time.time() - t1
        nb = -(-self.pairs // B)
        v = self.pairs / (self.n_frag * t_fcgf + nb * t_batch)
        return v, ("FCGF measured on %d of %d fragments (%.2fs each, C + OpenMP sparse-conv restatement, not ME) + "
                   "ONE timed 32-pair batch (%.2fs: 2x Soft_NN + OANet + diag_embed Kabsch, oracle/torch_port.py) "
                   "EXTRAPOLATED to the %d batches; scene rate = %d pairs / (%d x t_fcgf + %d x t_batch)"
                   % (nf, self.n_frag, t_fcgf, t_batch, nb, self.pairs, self.n_frag, nb)), \
            {"extrapolated": True, "fragments_timed": nf, "batches_timed": 1, "t_fcgf_s": round(t_fcgf, 3),
             "t_batch_s": round(t_batch, 3), "fcgf_backend": "C + OpenMP (oracle/csrc/sparse_conv.c)"}

    def fcgf_work(self):
        """Algorithmic work of one FCGF forward over the scene's fragments (lib/descriptor/fcgf.py:229-280), counted
        from the scene's kernel maps: FLOPs = 2 Cin Cout per (input, output) pair of every conv; compulsory bytes =
        input rows + output rows (+ residual rows) + weights + the neighbour table, fp32 / int32.  (Host syncs:
        call outside the timed region.)"""
        self._wait_prep()
        data = self.prepare()
        cm = data["sinput0_coords_manager"]
        M = {s: int(cm.coords_at(s).shape[0]) for s in (1, 2, 4, 8)}
        fl, by = 0.0, 0.0

        def conv(kind, s, ks, cin, cout, m_in, m_out, res=False):
            nonlocal fl, by
            if kind is None:
                pairs, K = m_out, 1
            else:
                nbr = cm.kernel_map(kind, s, ks)
                pairs, K = int((nbr >= 0).sum().item()), nbr.shape[1]
            fl += 2.0 * cin * cout * pairs
            by += 4.0 * (m_in * cin + m_out * cout * (2 if res else 1) + K * cin * cout) + (4.0 * m_out * K if kind else 0)

        def block(s, c):
            conv("s1", s, 3, c, c, M[s], M[s])
            conv("s1", s, 3, c, c, M[s], M[s], res=True)
        conv("s1", 1, 7, 1, 32, M[1], M[1])
        block(1, 32)
        conv("down", 1, 3, 32, 64, M[1], M[2]); block(2, 64)
        conv("down", 2, 3, 64, 128, M[2], M[4]); block(4, 128)
        conv("down", 4, 3, 128, 256, M[4], M[8]); block(8, 256)
        conv("up", 4, 3, 256, 128, M[8], M[4]); block(4, 128)
        conv("up", 2, 3, 256, 64, M[4], M[2]); block(2, 64)
        conv("up", 1, 3, 128, 64, M[2], M[1]); block(1, 64)
        conv(None, 1, 1, 96, 64, M[1], M[1])
        conv(None, 1, 1, 64, 32, M[1], M[1])
        return fl, by


def emulate_collectives():
    """--emulate-world: lib.distributed's collectives become local (rank 0 of N): an all-gather returns this rank's
    block repeated N times (the same bytes land, from a device copy instead of xGMI), the guard's MAX all-reduce keeps
    the local bit"""
    from lib import distributed as D

    def gather_rows(buf, world, pg=None):
        return buf.repeat((world,) + (1,) * (buf.dim() - 1))

    D.all_gather_rows = gather_rows
    D.all_reduce_max = lambda t, pg=None: None


def records_allgather(rec, world):
    import torch.distributed as dist
    from lib import distributed as D
    if not (dist.is_available() and dist.is_initialized()):
        return rec
    return D.all_gather_rows(rec.unsqueeze(0), world)


MFMA_CLASSES = ("conv_pts", "embed", "pool", "unpool", "oafilter", "feat_nn", "spconv", "pointcn")
# kernel classes with a split-fp16 form (switched together by lib/_native.set_math -> mvr_set_math)
F16_CLASSES = ("conv_pts", "embed", "pool", "unpool", "oafilter", "feat_nn", "spconv")


def _fcgf_mod():
    import lib.descriptor.fcgf as m
    return m


def _sparse_mod():
    import lib.sparse as m
    return m


def class_peak_tflops(cls, knobs):
    """fp32-equivalent MFMA peak of a kernel class at the arithmetic it runs: split-bf16 (6 products per fp32
    product) = 16 x 157.3 / 6 TF; split-fp16 (3 products) = 16 x 157.3 / 3 TF"""
    on = cls in F16_CLASSES and bool(knobs.get("split16"))
    return PEAK_BF16_TFLOPS / (3 if on else 6)


def timed_run(wl, args, world, pipelined, barrier):
    """warmup, one untimed profiled step (per-class breakdown, dominant class), the timed steps"""
    from lib import _native

    def run_step():
        if pipelined:
            return wl.step_pipelined(world)
        return wl.gather(wl.step(), world)

    with torch.no_grad():
        for _ in range(max(args.warmup, 1 if pipelined else 0)):   # the pipeline is filled before timing
            run_step()
        # one untimed step with events on every launch: the per-class breakdown and the dominant class;
        # the timed region then records events only around the dominant class's launches (events on
        # every launch cost ~1 ms per step).  --prof-seq (PMC attribution of exactly the timed steps'
        # launches) records every class in the timed region instead.
        prof_all, dom = None, None
        torch.cuda.synchronize()
        _native.prof_mask(None)
        if not args.prof_seq:
            _native.prof_set(1)
            wl.gather(wl.step(), world)   # stages back to back: per-class times without overlap
            torch.cuda.synchronize()
            prof_all = {k: _native.prof_get(k) for k in _native.PROF_KINDS}
            _native.prof_set(0)
            dom = max(prof_all, key=lambda k: prof_all[k][0])
            _native.prof_mask([dom])
        _native.prof_set(0 if args.no_prof else 1)
        barrier()
        torch.cuda.synchronize()
        # per-step boundaries for the median: an event on every stream a step enqueues on, recorded after the
        # step; step i ends when the last of them completes (events only, no host synchronisation per step)
        marks = wl.streams[:2] if pipelined else (torch.cuda.current_stream(),)
        ev0 = torch.cuda.Event(enable_timing=True)
        ev0.record(torch.cuda.current_stream())
        step_ev = []
        t0 = time.perf_counter()
        for _ in range(args.steps):
            rec = run_step()
            evs = []
            for st_ in marks:
                e = torch.cuda.Event(enable_timing=True)
                e.record(st_)
                evs.append(e)
            step_ev.append(evs)
        torch.cuda.synchronize()
        barrier()
        t1 = time.perf_counter()
        dt = t1 - t0
        ends = [max(ev0.elapsed_time(e) for e in evs) for evs in step_ev]
        step_ms = np.diff([0.0] + ends)
        prof = {k: _native.prof_get(k) for k in _native.PROF_KINDS}
        if prof_all is None:
            prof_all = {k: tuple(x / max(args.steps, 1) for x in v) for k, v in prof.items()}
            dom = max(prof, key=lambda k: prof[k][0])
        if args.prof_seq and int(os.environ.get("RANK", "0")) == 0:
            with open(args.prof_seq, "w") as f:
                json.dump(_native.prof_seq(), f)
        _native.prof_set(0)
        _native.prof_mask(None)
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():   # max over ranks
        from lib import distributed as D
        tt = torch.tensor([dt], device=rec.device, dtype=torch.float64)
        D.all_reduce_max(tt)
        dt = float(tt.item())
    return dt, rec, prof, prof_all, dom, step_ms


def _oanet_golden(dev, fx, seed, xs):
    from lib.filtering.oanet import OANet
    net = OANet(oanet_cfg())
    synth_module(net, seed=seed)
    net = net.to(dev).train()
    with torch.no_grad():
        out = net({"xs": torch.from_numpy(xs).to(dev).unsqueeze(1)})
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", fx)))
    return out, g


def _errs(out, ref, i, suffix=""):
    P = out["rot_est"][i].shape[0]
    dR = np.abs(out["rot_est"][i].cpu().numpy() - ref["R%d%s" % (i, suffix)]).reshape(P, -1).max(1)
    dt = np.abs(out["trans_est"][i].cpu().numpy() - ref["t%d%s" % (i, suffix)]).reshape(P, -1).max(1)
    return dR, dt


def golden_accuracy(dev):
    """R / t error of the OANet (RegBlock network, train-mode BN: the benchmark's mode) at the current maths, on
    full-size reference fixtures of 32 pairs x 5000 correspondences:
      * strict (headline): tests/golden/oanet_full_train_strict.npz, well conditioned (the reference's fp32 output
        within 1e-5 of the reference's own float64 output): per-block maxima vs the reference's fp32 and fp64
        outputs, the number of pairs over north_star's 1e-4 bound, mask mismatches away from 0.5;
      * stress: tests/golden/oanet_full_train.npz, chaotic in block 1 (the reference's own fp32 output sits up to
        2.6e-4 from exact arithmetic there; oanet_full_train_f64.npz = our float64 restatement)."""
    from synth import synth_correspondences
    g = dict(np.load(os.path.join(ROOT, "tests", "golden", "oanet_full_train_strict.npz")))
    p = json.loads(str(g["params"]))
    xs, _, _ = synth_correspondences(32, 5000, seed=p["xs_seed"], inlier_lo=p["inlier_lo"], inlier_hi=p["inlier_hi"])
    out, g = _oanet_golden(dev, "oanet_full_train_strict.npz", p["weights_seed"], xs)
    r = {"fixture": "oanet_full_train_strict.npz (32 pairs x 5000, train-mode BN, well conditioned)"}
    over = 0
    for i in range(2):
        for suffix, tag in (("", "ref"), ("_f64", "ref_f64")):
            dR, dt = _errs(out, g, i, suffix)
            r["block%d_max_R_err_vs_%s" % (i, tag)] = round(float(dR.max()), 8)
            r["block%d_max_t_err_vs_%s" % (i, tag)] = round(float(dt.max()), 8)
            if tag == "ref":
                over += int(((dR > 1e-4) | (dt > 1e-4)).sum())
    r["max_R_err_vs_ref"] = max(r["block%d_max_R_err_vs_ref" % i] for i in range(2))
    r["max_t_err_vs_ref"] = max(r["block%d_max_t_err_vs_ref" % i] for i in range(2))
    r["pair_blocks_over_1e-4"] = over
    r["mask_mismatches_vs_ref"] = sum(int(((out["scores"][i].cpu().numpy() > 0.5) != (g["scores%d" % i] > 0.5))
                                          [np.abs(g["scores%d" % i] - 0.5) >= 1e-4].sum()) for i in range(2))
    xs2, _, _ = synth_correspondences(32, 5000, seed=33)
    out2, g2 = _oanet_golden(dev, "oanet_full_train.npz", 7, xs2)
    g64 = dict(np.load(os.path.join(ROOT, "tests", "golden", "oanet_full_train_f64.npz")))
    st = {}
    for ref, tag in ((g2, "ref"), (g64, "f64_restatement")):
        st["max_R_err_vs_" + tag] = round(max(float(_errs(out2, ref, i)[0].max()) for i in range(2)), 8)
        st["max_t_err_vs_" + tag] = round(max(float(_errs(out2, ref, i)[1].max()) for i in range(2)), 8)
    st["ref_fp32_vs_f64_max"] = round(max(float(np.abs(g2[k % i] - g64[k % i]).max()) for i in range(2)
                                          for k in ("R%d", "t%d")), 8)
    r["stress"] = st
    return r


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--workload", default=os.environ.get("MVR_BENCH_WORKLOAD", "scene"),
                    choices=["scene", "precomputed"])
    ap.add_argument("--pairs", type=int, default=435)
    ap.add_argument("--frags", type=int, default=30,
                    help="scene workload: fragments per scene (30 = configs[2], a 3DMatch scene, 435 pairs; 50 = the "
                    "Redwood-scale scene of configs[4], 1225 pairs)")
    ap.add_argument("--npts", type=int, default=5000)
    ap.add_argument("--samp", default="rand", choices=["rand", "fps"],
                    help="scene workload: interest sampling (lib/layers.py Sampler: rand = the reference's numpy draws, "
                    "fps = furthest-point sampling, csrc/fps.hip)")
    ap.add_argument("--math", default=os.environ.get("MVR_MATH", "f32eq"), choices=["f32eq", "split16"],
                    help="f32eq: every MFMA product on the 3-term bf16 split (fp32-equivalent operands, the reference's "
                    "fp32); split16: the 2-term fp16 split (22-bit operands) where a kernel has it")
    ap.add_argument("--no-secondary", action="store_true", help="skip the secondary timed leg at the other maths")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=20.0)
    ap.add_argument("--no-prof", action="store_true", help="no per-launch HIP events in the timed region (A/B timing)")
    ap.add_argument("--no-pipeline", action="store_true", help="scene workload: run the stages of a step back to "
                    "back on one stream (default: two-stage pipeline over consecutive scenes, SceneWorkload.step_pipelined)")
    ap.add_argument("--shard", default=os.environ.get("MVR_BENCH_SHARD", "scenes"), choices=["scenes", "pairs"],
                    help="scene workload at N > 1: scenes = one scene per rank (weak scaling); pairs = ONE scene per "
                    "step, its fragments (FCGF + sampling) and its pair batch (feature NN + OANet + Procrustes) split "
                    "over the ranks, with an RCCL all-gather of the samples and of the per-pair records (strong scaling)")
    ap.add_argument("--emulate-world", type=int, default=0,
                    help="--shard pairs on ONE GPU: time rank 0 of an N-rank run (its fragments, its pair block; the "
                         "all-gathers and the guard all-reduce replaced by local copies of the same sizes) -- the "
                         "per-rank step of the N-GPU strong-scaling split, whose aggregate rate the line reports")
    ap.add_argument("--prof-seq", default=None, help="write the per-launch kernel-class sequence of the timed "
                    "steps (JSON) for PMC attribution (tools/pmc_traffic.py)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if os.environ.get("MVR_BENCH_BACKEND", "nccl") != "nccl":   # rehearsal: ranks may share the box's GPUs
        local %= max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # MVR_BENCH_PG=1: the RCCL process group (barriers, record all-gather) also at one rank, to exercise the N > 1
    # data path on a one-GPU box
    use_pg = world > 1 or os.environ.get("MVR_BENCH_PG") == "1"
    # MVR_BENCH_BACKEND=gloo: several ranks on one GPU (a rehearsal of the N > 1 paths on a one-GPU box; RCCL
    # refuses two ranks on one device): the collectives are staged through host memory (lib/distributed.py)
    backend = os.environ.get("MVR_BENCH_BACKEND", "nccl")
    groups = None
    if use_pg:
        import torch.distributed as dist
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29517")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev, rank=rank, world_size=world)
        else:
            dist.init_process_group(backend, rank=rank, world_size=world)
        if args.shard == "pairs" and args.workload == "scene":
            # voxel counts (host, gloo) | sampled descriptors (stream A) | filter guard + records (stream B): one
            # communicator per stream, so the two streams' collectives never queue behind each other
            groups = (dist.new_group(backend="gloo"), dist.new_group(backend=backend),
                      dist.group.WORLD)

    def barrier():
        if use_pg:
            import torch.distributed as dist
            dist.barrier()

    from lib import _native
    _native.lib()
    math_info = _native.set_math(args.math)
    emulate = args.emulate_world > 1
    if emulate:
        if world > 1 or args.shard != "pairs":
            raise SystemExit("--emulate-world runs one process with --shard pairs")
        emulate_collectives()
        world = args.emulate_world
    if args.workload == "scene":
        if args.shard == "pairs" and not use_pg and not emulate:
            raise SystemExit("--shard pairs needs a process group (torchrun, or MVR_BENCH_PG=1 at one rank)")
        if args.shard == "pairs" and world > args.frags:
            raise SystemExit("--shard pairs: at most one rank per fragment (%d)" % args.frags)
        wl = SceneWorkload(dev, rank, npts=args.npts, n_frag=args.frags, samp=args.samp, shard=args.shard,
                           world=world, groups=groups or (None, None, None), emulate=emulate)
    else:
        wl = PrecomputedWorkload(dev, rank, args.pairs, args.npts, shard=args.shard, world=world)
    pipelined = args.workload == "scene" and not args.no_pipeline

    dt, rec, prof, prof_all, dom, step_ms = timed_run(wl, args, world, pipelined, barrier)
    pair_sharded = args.shard == "pairs"
    pairs_per_step = int(rec.shape[0]) if pair_sharded else int(rec.shape[-2]) * world
    value = pairs_per_step * args.steps / dt
    ms_step = dt / args.steps * 1e3

    # FCGF sparse convs: the launch-level ProfScope cannot see how many kernel-map pairs a launch has (no host
    # sync); the class's algorithmic FLOPs / bytes are counted here from the scene's kernel maps instead
    fcgf = None
    if args.workload == "scene":
        fl, by = wl.fcgf_work()
        fcgf = {"flops_per_step": fl, "bytes_per_step": by}
        for d in (prof_all, prof):
            if d.get("spconv") and d["spconv"][1]:
                scale = 1.0 if d is prof_all else float(args.steps)
                d["spconv"] = (d["spconv"][0], d["spconv"][1], fl * scale, by * scale)

    # dominant kernel class (by device time in the profiled untimed step), timed with HIP events around
    # each of its launches inside the timed region and priced against the roofline that binds it:
    # arithmetic intensity vs the ridge of the MFMA path it runs on
    knobs = math_info["knobs"]
    ms, nl, fl, by = prof[dom]
    if ms <= 0:   # --no-prof: no per-launch timings
        ms, nl = 1e-9, 1
    mpeak = class_peak_tflops(dom, knobs) if dom in MFMA_CLASSES else PEAK_FP32_TFLOPS
    ridge = mpeak * 1e12 / (PEAK_HBM_GBS * 1e9)                     # FLOP per byte
    bound = "mfma" if (by > 0 and fl / by >= ridge) else "hbm"
    avg_s = ms * 1e-3 / max(nl, 1)
    if bound == "mfma":
        achieved, peak, unit = fl / max(nl, 1) / avg_s / 1e12, mpeak, "TFLOP/s"
    else:
        achieved, peak, unit = by / max(nl, 1) / avg_s / 1e9, PEAK_HBM_GBS, "GB/s"
    traffic, tsrc = None, None
    tfile = os.environ.get("MVR_PMC_TRAFFIC", os.path.join(ROOT, "profiles", "pmc_traffic.json"))
    tnote = "no PMC file"
    if os.path.exists(tfile):
        with open(tfile) as f:
            tr = json.load(f)
        have = _native.source_hash()
        if tr.get("lib_hash") != have:
            # counters of another build (e.g. a previous round's kernels) never price this one
            tnote = "PMC file is of library %s, this run loads %s: traffic not measured for this build" % (
                tr.get("lib_hash"), have)
        elif tr.get("math", "split16") != args.math:
            tnote = "PMC file measured --math %s" % tr.get("math")
        elif dom in tr.get("classes", {}):
            traffic = tr["classes"][dom]["pmc_bytes_per_launch"]
            tsrc = tr.get("source")
            tnote = "PMC of this library (%s)" % have
    # the same kernel class alone on the GPU (the untimed profiled step runs the stages back to back):
    # in the pipelined timed region its launches share the chip with the other stream's kernels
    iso = prof_all.get(dom, (0.0, 0, 0.0, 0.0))
    iso_ach = None
    if iso[0] > 0 and iso[1]:
        iso_s = iso[0] * 1e-3 / iso[1]
        iso_ach = (iso[2] / iso[1] / iso_s / 1e12) if bound == "mfma" else (iso[3] / iso[1] / iso_s / 1e9)
    # SURVEY §8d whole-step roofline: T_floor = sum over kernel classes of max(FLOP / MFMA peak at the class's
    # arithmetic, algorithmic bytes / 8 TB/s), per step, against the measured step time
    floor_ms = {}
    for k, v in prof_all.items():
        if not v[1]:
            continue
        pk = class_peak_tflops(k, knobs) if k in MFMA_CLASSES else PEAK_FP32_TFLOPS
        floor_ms[k] = 1e3 * max(v[2] / (pk * 1e12), v[3] / (PEAK_HBM_GBS * 1e9))
    t_floor = sum(floor_ms.values())
    roof = {"bound": bound, "achieved": round(achieved, 3), "peak": round(peak, 1), "unit": unit,
            "frac": round(achieved / peak, 4), "traffic": traffic,
            "achieved_isolated": round(iso_ach, 3) if iso_ach else None,
            "frac_isolated": round(iso_ach / peak, 4) if iso_ach else None,
            "kernel": dom, "launches_per_step": nl / max(args.steps, 1),
            "avg_launch_ms": round(ms / max(nl, 1), 4), "share_of_step": round(ms / (dt * 1e3), 3),
            "arith_intensity": round(fl / by, 2) if by else None, "ridge": round(ridge, 1),
            "algorithmic_bytes_per_launch": by / max(nl, 1),
            "peak_note": ("fp32-equivalent MFMA peak of the class's operand split (split-bf16 16*157.3/6 TF, "
                          "split-fp16 16*157.3/3 TF); HBM 8 TB/s (MI355X_MICROARCH.md)"),
            "traffic_source": tsrc, "traffic_note": tnote,
            # per kernel class, from the profiled untimed step (events on every launch):
            # [ms per step, algorithmic TFLOP/s, algorithmic GB/s]
            "classes": {k: [round(v[0], 3), round(v[2] / (v[0] * 1e9), 1), round(v[3] / (v[0] * 1e6))]
                        for k, v in prof_all.items() if v[1] and v[0] > 0},
            "whole_step": {"t_floor_ms": round(t_floor, 3), "ms_per_step": round(ms_step, 3),
                           "achieved": round(t_floor / ms_step, 4),
                           "floor_ms_by_class": {k: round(v, 3) for k, v in floor_ms.items()},
                           "note": "SURVEY §8d: T_floor = sum over classes of max(FLOP / MFMA peak at the class's "
                                   "operand split, algorithmic bytes / 8 TB/s); achieved = T_floor / measured step"},
            "fcgf_work": fcgf}

    # the other operand maths as a secondary line (same workload, same step count), and the accuracy of both on
    # the full-size golden
    secondary, accuracy = None, None
    if not args.no_secondary and args.workload == "scene":
        other = "split16" if args.math == "f32eq" else "f32eq"
        oinfo = _native.set_math(other)
        odt, orec, _, _, _, ostep = timed_run(wl, args, world, pipelined, barrier)
        if rank == 0:
            acc_o = golden_accuracy(dev)
        _native.set_math(args.math)
        secondary = {"math": other, "dtype": oinfo["dtype"], "value": round(pairs_per_step * args.steps / odt, 3),
                     "ms_per_step": round(odt / args.steps * 1e3, 3),
                     "ms_per_step_median": round(float(np.median(ostep)), 3)}
        if rank == 0:
            secondary["accuracy"] = acc_o
    if rank == 0:
        accuracy = golden_accuracy(dev)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        # the box's CPU share per GPU (OMP_NUM_THREADS is set to it there; affinity shows the whole host)
        cores = int(os.environ.get("OMP_NUM_THREADS", "0")) or len(os.sched_getaffinity(0))
        v, sample, extra = wl.cpu_baseline(cores, args.cpu_budget)
        v8, _, _ = wl.cpu_baseline(8, args.cpu_budget)
        cpu = dict({"value": round(v, 4), "unit": "pairs/s", "cores": cores, "kind": "port", "sample": sample,
                    "value_8_threads": round(v8, 4)}, **extra)
        if args.workload == "scene":   # the instruction set of the C sparse conv on this host (oracle/csrc clone)
            from oracle.fcgf import isa
            cpu["fcgf_isa"] = isa()
    line = {"metric": METRIC if args.workload == "scene" else METRIC + " [filter+SVD only: precomputed corr.]",
            "value": round(value, 3), "unit": "pairs/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_step, 3),
            "ms_per_step_median": round(float(np.median(step_ms)), 3),
            "ms_per_step_min_max": [round(float(step_ms.min()), 3), round(float(step_ms.max()), 3)],
            "higher_is_better": True,
            "scaling": "strong" if pair_sharded else "weak", "vs_baseline": None, "dtype": math_info["dtype"], "data": "synthetic",
            "config": dict(wl.config(), math=args.math,
                           oanet_point_layout={1: "chunk-major", 0: "row-major"}.get(
                               _native.lib().mvr_oan_last_layout(), "none"),
                           emulated=("rank 0 of %d on ONE GPU: collectives replaced by local copies of the same "
                                     "sizes; value = the whole job's pairs / rank 0's step" % world) if emulate else None,
                           spconv_presplit_planes=bool(_fcgf_mod().PRESPLIT), spatial_map_order=bool(
                               _sparse_mod().SPATIAL_MAPS), library=_native.source_hash(),
                           parallelism=(("pairs%d (one scene per step: fragments and pair batch sharded over %d "
                                         "ranks, %s all-gather of samples and records)"
                                         if args.workload == "scene" else
                                         "pairs%d (one evaluation per step: its 32-pair loader batches in contiguous "
                                         "blocks over %d ranks, %s all-gather of the records)")
                                        % (world, world, "RCCL" if backend == "nccl" else backend)
                                        if pair_sharded else
                                        "dp%d (one scene per rank, %s all-gather of records)"
                                        % (world, "RCCL" if backend == "nccl" else backend)),
                           schedule=("3-stream pipeline over consecutive scenes: voxelisation + coordinate levels of "
                                     "scene k+1, FCGF + feature NN of scene k, OANet + Procrustes of scene k-1; every "
                                     "timed step runs every stage in full"
                                     if pipelined else "stages back to back on one stream")),
            "roofline": roof, "cpu_baseline": cpu, "accuracy": accuracy, "secondary": secondary}
    if rank == 0:
        print(json.dumps(line), flush=True)
    if use_pg:
        import torch.distributed as dist
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
