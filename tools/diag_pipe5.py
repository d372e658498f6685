"""Intermittent pipelined-vs-sequential difference hunt: many pipelined scene steps, each stage's output
compared with the sequential reference ON ITS OWN STREAM right after it is produced (only small diff
scalars are kept, so buffer lifetimes are the bench's).  usage: python tools/diag_pipe5.py [steps]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import torch  # noqa: E402
import bench  # noqa: E402


def main():
    steps = int(sys.argv[1]) if len(sys.argv) > 1 else 30
    npts = int(sys.argv[2]) if len(sys.argv) > 2 else 1000
    nfrag = int(sys.argv[3]) if len(sys.argv) > 3 else 4
    dev = torch.device("cuda")
    wl = bench.SceneWorkload(dev, 0, npts=npts, n_frag=nfrag)
    ref = {}
    orig_desc = wl.describe
    diffs = []

    def finish(fin):
        xs = fin["xs"]
        out = wl.model.filter_correspondences(fin)
        lg = out["logits"][-1]
        R, t, s = out["rot_est"][-1], out["trans_est"][-1], out["scores"][-1]
        rec = torch.cat([R.reshape(-1, 9), t.reshape(-1, 3), (s > 0.5).float().mean(dim=1, keepdim=True)], 1)
        if "xs" not in ref:
            ref.update(xs=xs.clone(), lg=lg.clone(), rec=rec.clone())
        else:
            diffs.append(("B", torch.stack([(xs - ref["xs"]).abs().max(), (lg - ref["lg"]).abs().max(),
                                            (rec - ref["rec"]).abs().max()])))
        return rec

    def describe():
        fin = orig_desc()
        if "x" not in ref:
            ref.update(x=fin["xs"].clone())
        else:
            diffs.append(("A", torch.stack([(fin["xs"] - ref["x"]).abs().max()])))
        return fin

    wl.finish, wl.describe = finish, describe
    with torch.no_grad():
        wl.step()
        torch.cuda.synchronize()
        for _ in range(steps):
            wl.step_pipelined(1)
    torch.cuda.synchronize()
    nbad = 0
    for i, (k, v) in enumerate(diffs):
        v = v.tolist()
        if any(x != 0 for x in v):
            nbad += 1
            print(i, k, ["%.3g" % x for x in v], flush=True)
    print("stage outputs compared: %d, differing: %d" % (len(diffs), nbad))


if __name__ == "__main__":
    main()
