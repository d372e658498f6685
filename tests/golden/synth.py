"""Deterministic synthetic parameters and inputs shared by the golden-vector
generator (`make_golden.py`, which runs the *reference* modules in this
container) and the parity tests (which run our HIP path and the oracle).

Nothing here imports the reference.  Every array is a pure function of
(name, shape, seed) so fixtures only need to store inputs/outputs, never the
2.4 M OANet parameters.
"""
import zlib

import numpy as np


def _rng(name, seed):
    return np.random.RandomState((zlib.crc32(name.encode()) + 7919 * seed) % (2 ** 31))


def synth_state(shapes, seed=0, overrides=None):
    """Build a state dict {name: np.ndarray} for the given {name: shape}.

    Conv weights  ~ N(0, 1/fan_in)      (keeps activations O(1) through 12 layers)
    conv biases   ~ N(0, 0.05)
    BN weight     ~ U(0.6, 1.4), BN bias ~ N(0, 0.1)
    BN running_mean ~ N(0, 0.2), running_var ~ U(0.5, 2.0)
    num_batches_tracked = 0
    """
    out = {}
    for name, shape in shapes.items():
        shape = tuple(shape)
        r = _rng(name, seed)
        if name.endswith("num_batches_tracked"):
            out[name] = np.zeros(shape, dtype=np.int64)
            continue
        base = name.rsplit(".", 1)[0]
        wshape = shapes.get(base + ".weight")
        is_conv = wshape is not None and len(wshape) >= 2
        if name.endswith(".kernel"):                      # MinkowskiEngine conv [K, Cin, Cout]
            fan_in = int(shape[0] * shape[1])
            out[name] = (r.standard_normal(shape) * np.sqrt(2.0 / fan_in)).astype(np.float32)
        elif name.endswith(".weight") and len(shape) >= 2:
            fan_in = int(np.prod(shape[1:]))
            out[name] = (r.standard_normal(shape) / np.sqrt(fan_in)).astype(np.float32)
        elif name.endswith(".bias") and is_conv:
            out[name] = (0.05 * r.standard_normal(shape)).astype(np.float32)
        elif name.endswith(".weight"):
            out[name] = r.uniform(0.6, 1.4, shape).astype(np.float32)
        elif name.endswith(".bias"):
            out[name] = (0.1 * r.standard_normal(shape)).astype(np.float32)
        elif name.endswith("running_mean"):
            out[name] = (0.2 * r.standard_normal(shape)).astype(np.float32)
        elif name.endswith("running_var"):
            out[name] = r.uniform(0.5, 2.0, shape).astype(np.float32)
        elif name.endswith("_temperature"):
            out[name] = np.asarray(0.3, dtype=np.float32).reshape(shape)
        else:
            out[name] = (0.1 * r.standard_normal(shape)).astype(np.float32)
    if overrides:
        for k, v in overrides.items():
            out[k] = np.asarray(v, dtype=out[k].dtype).reshape(out[k].shape) if k in out else v
    return out


def synth_correspondences(P, N, seed=0, inlier_lo=0.05, inlier_hi=0.4):
    """Synthetic putative correspondences xs [P, N, 6] in the shape of the
    precomputed-correspondence benchmark input:
    x1 uniform in a 3 m box, an inlier fraction maps through a random rigid
    motion with clipped noise (cf. lib/utils.py:390-415), the rest are outliers.
    Returns xs (float32) and the GT (R, t)."""
    r = np.random.RandomState(seed)
    xs = np.empty((P, N, 6), dtype=np.float32)
    Rs = np.empty((P, 3, 3), dtype=np.float32)
    ts = np.empty((P, 3), dtype=np.float32)
    for p in range(P):
        q = r.standard_normal(4)
        q /= np.linalg.norm(q)
        w, x, y, z = q
        R = np.array([
            [1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
            [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
            [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])
        t = r.standard_normal(3)
        x1 = r.uniform(-1.5, 1.5, (N, 3))
        frac = r.uniform(inlier_lo, inlier_hi)
        inl = r.rand(N) < frac
        x2 = r.uniform(-1.5, 1.5, (N, 3)) + t
        noise = np.clip(0.01 * r.standard_normal((N, 3)), -0.025, 0.025)
        x2[inl] = (x1[inl] @ R.T) + t + noise[inl]
        xs[p, :, :3] = x1
        xs[p, :, 3:] = x2
        Rs[p] = R
        ts[p] = t
    return xs, Rs, ts


def unit_features(B, N, C, seed=0):
    r = np.random.RandomState(seed)
    f = r.standard_normal((B, N, C)).astype(np.float32)
    f /= np.linalg.norm(f, axis=-1, keepdims=True)
    return f.astype(np.float32)


# ----------------------------------------------------------------------------- synthetic scenes
def _rect(o, u, v):
    return (np.asarray(o, float), np.asarray(u, float), np.asarray(v, float))


def synth_room(seed=41, n_boxes=12, size=(6.0, 6.0, 3.0)):
    """Axis-aligned room (floor, ceiling, 4 walls) + boxes on the floor, as rectangles
    (origin, edge u, edge v) (SURVEY §8d synthetic 3DMatch-like scene)."""
    r = np.random.default_rng(seed)
    X, Y, Z = size
    rects = [_rect((0, 0, 0), (X, 0, 0), (0, Y, 0)), _rect((0, 0, Z), (X, 0, 0), (0, Y, 0)),
             _rect((0, 0, 0), (X, 0, 0), (0, 0, Z)), _rect((0, Y, 0), (X, 0, 0), (0, 0, Z)),
             _rect((0, 0, 0), (0, Y, 0), (0, 0, Z)), _rect((X, 0, 0), (0, Y, 0), (0, 0, Z))]
    for _ in range(n_boxes):
        w, d, h = r.uniform(0.3, 1.2, 3)
        x0, y0 = r.uniform(0.2, X - 0.2 - w), r.uniform(0.2, Y - 0.2 - d)
        rects += [_rect((x0, y0, h), (w, 0, 0), (0, d, 0)),
                  _rect((x0, y0, 0), (w, 0, 0), (0, 0, h)), _rect((x0, y0 + d, 0), (w, 0, 0), (0, 0, h)),
                  _rect((x0, y0, 0), (0, d, 0), (0, 0, h)), _rect((x0 + w, y0, 0), (0, d, 0), (0, 0, h))]
    return rects


def sample_rects(rects, density, rng):
    pts = []
    for o, u, v in rects:
        n = int(np.linalg.norm(np.cross(u, v)) * density)
        a = rng.random((n, 2))
        pts.append(o + a[:, :1] * u + a[:, 1:] * v)
    return np.concatenate(pts)


def random_rotation(rng):
    q = rng.standard_normal(4)
    q /= np.linalg.norm(q)
    w, x, y, z = q
    return np.array([[1 - 2 * (y * y + z * z), 2 * (x * y - z * w), 2 * (x * z + y * w)],
                     [2 * (x * y + z * w), 1 - 2 * (x * x + z * z), 2 * (y * z - x * w)],
                     [2 * (x * z - y * w), 2 * (y * z + x * w), 1 - 2 * (x * x + y * y)]])


def synth_scene_fragments(n_frag=30, seed=41, n_pts=250000, density=26000.0):
    """n_frag raw fragments of one synthetic room: camera random walk (0.3 m steps), the
    n_pts surface points nearest to the camera (at this density 250k points cover
    ~20k 2.5 cm voxels, like the demo fragment's 258k points -> 19k voxels), each
    moved by a random SE(3).
    Returns (list of float32 [n,3], list of 4x4 GT poses mapping fragment -> world)."""
    rng = np.random.default_rng(seed)
    scene = sample_rects(synth_room(seed), density, rng)
    cam = np.array([3.0, 3.0, 1.5])
    frags, poses = [], []
    for _ in range(n_frag):
        cam = np.clip(cam + rng.normal(0, 0.3, 3) * np.array([1, 1, 0.3]), [1.0, 1.0, 1.2], [5.0, 5.0, 1.8])
        d = np.linalg.norm(scene - cam, axis=1)
        sel = np.argpartition(d, n_pts)[:n_pts] if len(d) > n_pts else np.arange(len(d))
        R = random_rotation(rng)
        t = rng.normal(0, 1.0, 3)
        p = (scene[sel] - cam) @ R.T + t             # fragment frame
        T = np.eye(4)                                  # fragment -> world: x_w = R^T (x_f - t) + cam
        T[:3, :3] = R.T
        T[:3, 3] = cam - R.T @ t
        frags.append(p.astype(np.float32))
        poses.append(T)
    return frags, poses
