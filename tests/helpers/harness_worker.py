"""One rank of the multi-process evaluation-harness tests (tests/test_harness_distributed.py on CPU,
tests/test_gpu_harness_distributed.py on the box's GPU): scripts/benchmark_pairwise_registration.main(argv) under
torchrun's environment (RANK / WORLD_SIZE / MASTER_*), gloo process group.  Writes this rank's returned summary to
<out>/summary_<rank>.json.

usage: RANK=r WORLD_SIZE=w MASTER_ADDR=127.0.0.1 MASTER_PORT=p python harness_worker.py <out> <cwd> [stub] -- argv..."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
for p in (os.path.join(ROOT, "3d_multiview_reg_amd"), ROOT, os.path.join(ROOT, "tests", "golden"), HERE):
    if p not in sys.path:
        sys.path.insert(0, p)


def stub_batch_records(batch, bi, method, model, refine, seed, overlap_method, overlap_threshold):
    """CPU stand-in for the harness's per-batch GPU work (filter / RANSAC + overlap gate): a deterministic function
    of the batch's correspondences, its global batch index and the pair index, in the harness's record layout"""
    import numpy as np
    from scripts.benchmark_pairwise_registration import REC
    xs = batch["xs"][:, 0].double().numpy()
    b = xs.shape[0]
    rec = np.zeros((b, REC), np.float64)
    for k in range(b):
        T = np.eye(4)
        T[:3, 3] = xs[k, :, 3:].mean(0) - xs[k, :, :3].mean(0) + 1e-3 * bi
        meta = batch["metadata"][k]
        p = int(batch["idx"][k].numpy().item())
        rec[k, 0] = p
        rec[k, 1:17] = T.reshape(16)
        rec[k, 17] = float((p + bi) % 3 != 0)
        rec[k, 18], rec[k, 19] = int(meta[1]), int(meta[2])
    return rec


def main():
    sep = sys.argv.index("--")
    out, cwd = sys.argv[1], sys.argv[2]
    stub = len(sys.argv[3:sep]) > 0 and sys.argv[3] == "stub"
    argv = sys.argv[sep + 1:]
    os.chdir(cwd)
    import scripts.benchmark_pairwise_registration as H
    if stub:
        H._batch_records = stub_batch_records
    s = H.main(argv)
    with open(os.path.join(out, "summary_%s.json" % os.environ.get("RANK", "0")), "w") as f:
        json.dump(s, f, sort_keys=True)
    import torch.distributed as dist
    if dist.is_initialized():
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
