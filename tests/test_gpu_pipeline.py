"""The bench's two-stage stream pipeline (bench.py SceneWorkload.step_pipelined: OANet + Procrustes of
scene k-1 on one HIP stream while scene k is voxelised, described by FCGF and matched on another) returns the same
per-pair records as the stages run back to back on one stream — bit for bit, every kernel on the path is
run-to-run deterministic — and no forward pass blocks the host (the SVD-fallback flag stays on the device
until read)."""
import pytest

pytestmark = pytest.mark.gpu


def test_pipelined_scene_records_equal_sequential(gpu):
    import torch
    import bench
    wl = bench.SceneWorkload(gpu, 0, npts=1000, n_frag=4)
    with torch.no_grad():
        ref = [wl.step() for _ in range(2)]
        assert wl.step_pipelined(1) is None          # fills the pipeline
        got = [wl.step_pipelined(1) for _ in range(2)]
    torch.cuda.synchronize()
    assert ref[0].shape == (6, 13)
    assert torch.equal(ref[0], ref[1])
    for i, g in enumerate(got):
        bad = (g != ref[0]).any(dim=1).nonzero().flatten().tolist()
        assert not bad, (i, bad, (g - ref[0]).abs().max().item())


def test_oanet_forward_does_not_block_the_host(gpu):
    import numpy as np
    import torch
    from synth import synth_state, synth_correspondences
    from lib.filtering.oanet import OANet, DeviceFlag
    cfg = {"misc": {"net_depth": 12, "clusters": 64, "iter_num": 1, "net_channel": 64, "use_gpu": True,
                    "normalize_weights": True}, "data": {"use_mutuals": 0}}
    net = OANet(cfg)
    st = synth_state({k: tuple(v.shape) for k, v in net.state_dict().items()}, seed=1)
    net.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in st.items()})
    net = net.to(gpu).eval()
    xs, _, _ = synth_correspondences(3, 1000, seed=2)
    with torch.no_grad():
        out = net({"xs": torch.from_numpy(xs).unsqueeze(1)})
    assert isinstance(out["gradient_flag"], DeviceFlag)
    assert out["gradient_flag"] == False  # noqa: E712  (reads the device flag)
    assert not out["gradient_flag"]


def test_full_scene_pipelined_equals_sequential(gpu):
    """The bench's own configuration (30 fragments, 5000 samples, 435 pairs): the pipelined step's records
    equal the sequential ones bit for bit (the full size is where cross-workgroup and cross-stream timing
    differ; the small scene above cannot show an order- or timing-dependent kernel)."""
    import torch
    import bench
    wl = bench.SceneWorkload(gpu, 0)
    with torch.no_grad():
        ref = wl.step()
        wl.step_pipelined(1)
        got = [wl.step_pipelined(1) for _ in range(3)]
    torch.cuda.synchronize()
    assert ref.shape == (435, 13)
    for g in got:
        assert torch.equal(g, ref), (g - ref).abs().max().item()


def test_redwood_scale_scene_pipelined_equals_sequential(gpu):
    """BASELINE configs[4]'s scene size (a Redwood-scale scene of 50 fragments -> 1,225 pairs, bench.py --frags 50):
    the pipelined records equal the sequential ones bit for bit, every pair registered (finite R, t)"""
    import torch
    import bench
    wl = bench.SceneWorkload(gpu, 0, n_frag=50)
    with torch.no_grad():
        ref = wl.step()
        wl.step_pipelined(1)
        got = [wl.step_pipelined(1) for _ in range(2)]
    torch.cuda.synchronize()
    assert ref.shape == (1225, 13)
    assert torch.isfinite(ref).all()
    for g in got:
        assert torch.equal(g, ref), (g - ref).abs().max().item()


def test_precomputed_pair_sharded_blocks_equal_whole(gpu):
    """bench.py --workload precomputed --shard pairs: each rank's block of whole 32-pair batches (here every block
    of a 3-rank split, run one after another in this process) gives exactly the whole evaluation's records"""
    import torch
    import bench
    whole = bench.PrecomputedWorkload(gpu, 0, 100, 5000, shard="pairs", world=1)
    with torch.no_grad():
        ref = whole.step()
        parts = [bench.PrecomputedWorkload(gpu, r, 100, 5000, shard="pairs", world=3).step() for r in range(3)]
    torch.cuda.synchronize()
    assert [p.shape[0] for p in parts] == [64, 36, 0]           # rank 2: an empty block
    assert torch.equal(torch.cat(parts), ref)


def test_oanet_full_size_stage_hashes_repeat(gpu):
    """Every intermediate activation and statistics buffer of the two OANet blocks (mvr_debug_stage_hash:
    ~110 stages at 435 pairs x 5000 points) is bit-identical over repeated forwards."""
    import torch
    import bench
    from lib import _native as NV
    wl = bench.PrecomputedWorkload(gpu, 0, 435, 5000)
    L = NV.lib()
    hs = []
    with torch.no_grad():
        for _ in range(4):
            buf = torch.zeros(256, dtype=torch.int64, device=gpu)
            L.mvr_debug_stage_hash(NV.ptr(buf), 256)
            try:
                wl.step()
            finally:
                L.mvr_debug_stage_hash(None, 0)
            hs.append(buf)
    torch.cuda.synchronize()
    n = int((hs[1] != 0).sum())
    assert n > 100
    # run 0 hashes never-written halves of shared statistics buffers before their first producer ran
    for h in hs[2:]:
        assert torch.equal(h, hs[1])
