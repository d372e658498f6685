"""The 3DMatch / Redwood evaluation harness (lib/utils.py mirror of /root/reference/lib/utils.py:438-637) against
the reference's own outputs: tests/golden/evalharness.npz holds the trajectory text the reference's
write_trajectory produced, what its read_trajectory / read_trajectory_info returned, extract_corresponding_trajectors,
computeTransformationErr per GT pair and evaluate_registration's precision / recall at two thresholds (including its
quirk that GT row 0, a non-consecutive pair here, is never counted).  nibabel is absent: the fixture's mat2quat is
tests/golden/make_golden.py's restatement, so the quaternion step itself stays parity-unpinned."""
import numpy as np

from conftest import golden
from lib.utils import (computeTransformationErr, evaluate_registration, extract_corresponding_trajectors,
                       read_trajectory, read_trajectory_info, write_trajectory)


def _meta(g):
    return np.asarray([[str(i), str(j), f] for (i, j), f in zip(g["est_pairs"], g["flags"])])


def test_write_trajectory_text(tmp_path):
    g = golden("evalharness.npz")
    p = tmp_path / "traj.txt"
    write_trajectory(g["est_T"], _meta(g), str(p))
    assert p.read_text() == str(g["traj_txt"])
    # the benchmark stores a bool flag; the mirror writes the same text for it (the reference writes nothing)
    mb = [[str(i), str(j), f == "True"] for (i, j), f in zip(g["est_pairs"], g["flags"])]
    q = tmp_path / "traj_bool.txt"
    write_trajectory(g["est_T"], mb, str(q))
    assert q.read_text() == str(g["traj_txt"])
    r = tmp_path / "gt.log"
    write_trajectory(g["gt_T"], [[str(i), str(j), "True"] for i, j in g["gt_pairs"]], str(r))
    assert r.read_text() == str(g["gt_txt"])


def test_read_trajectory_and_info(tmp_path):
    g = golden("evalharness.npz")
    p = tmp_path / "traj.txt"
    p.write_text(str(g["traj_txt"]))
    keys, traj = read_trajectory(str(p))
    np.testing.assert_array_equal(keys, g["keys"])
    np.testing.assert_array_equal(traj, g["traj_read"])
    i = tmp_path / "gt.info"
    i.write_text(str(g["info_txt"]))
    n, info = read_trajectory_info(str(i))
    assert n == int(g["n_frame"])
    np.testing.assert_array_equal(info, g["info_read"])


def test_corresponding_trajectories_and_metrics():
    g = golden("evalharness.npz")
    est, gt = extract_corresponding_trajectors(g["keys"], g["gt_keys"], g["traj_read"], g["gt_read"])
    np.testing.assert_array_equal(est, g["ext_est"])
    np.testing.assert_array_equal(gt, g["ext_gt"])
    for k, (i, j) in enumerate(g["gt_pairs"]):
        e = [n for n in range(len(g["est_pairs"])) if tuple(g["est_pairs"][n]) == (i, j)][0]
        err = computeTransformationErr(np.linalg.inv(g["gt_T"][k]) @ g["est_T"][e], g["gt_info"][k])
        np.testing.assert_allclose(err, g["errs"][k], rtol=1e-9, atol=1e-15)
    for err2 in (0.2, 0.05):
        p, r = evaluate_registration(int(g["n_frame"]), g["traj_read"], g["keys"], g["gt_keys"], g["gt_read"],
                                     g["info_read"], err2=err2)
        assert p == float(g["precision_%g" % err2]) and r == float(g["recall_%g" % err2])
