"""OANet inlier-weight network restated in numpy (TEST ORACLE ONLY).

Follows /root/reference/lib/filtering/oanet.py op for op.  Activations are
kept as [B, C, N] (the reference's [B, C, N, 1] without the trailing 1).
Weights come from a state dict with the reference's key names
(e.g. 'reg_init.l1_1.0.conv.3.weight').
"""
import numpy as np

from .kabsch import kabsch


class _Ctx:
    def __init__(self, state, train, dtype):
        self.s = state
        self.train = train
        self.dt = dtype

    def p(self, k):
        return np.asarray(self.s[k], dtype=self.dt)


def instance_norm(x, eps):
    """nn.InstanceNorm2d(C, eps) default affine=False: per (b, c) over N, biased var."""
    m = x.mean(axis=2, keepdims=True)
    v = ((x - m) ** 2).mean(axis=2, keepdims=True)
    return (x - m) / np.sqrt(v + x.dtype.type(eps))


def batch_norm(ctx, x, pre, eps=1e-5):
    """nn.BatchNorm2d(C): eval -> running stats; train -> batch stats over (B, N), biased var."""
    g, b = ctx.p(pre + ".weight"), ctx.p(pre + ".bias")
    if ctx.train:
        m = x.mean(axis=(0, 2), keepdims=True)
        v = ((x - m) ** 2).mean(axis=(0, 2), keepdims=True)
    else:
        m = ctx.p(pre + ".running_mean")[None, :, None]
        v = ctx.p(pre + ".running_var")[None, :, None]
    return (x - m) / np.sqrt(v + x.dtype.type(eps)) * g[None, :, None] + b[None, :, None]


def conv1x1(ctx, x, pre):
    """nn.Conv2d(Cin, Cout, 1) on [B, Cin, N]."""
    W = ctx.p(pre + ".weight")[:, :, 0, 0]
    y = np.matmul(W[None], x)
    if pre + ".bias" in ctx.s:
        y = y + ctx.p(pre + ".bias")[None, :, None]
    return y


def relu(x):
    return np.maximum(x, 0)


def pointcn(ctx, x, pre):
    """oanet.py:18-43 PointCN: IN(1e-5) BN ReLU Conv IN BN ReLU Conv (+ shot_cut or identity)."""
    o = relu(batch_norm(ctx, instance_norm(x, 1e-5), pre + ".conv.1"))
    o = conv1x1(ctx, o, pre + ".conv.3")
    o = relu(batch_norm(ctx, instance_norm(o, 1e-5), pre + ".conv.5"))
    o = conv1x1(ctx, o, pre + ".conv.7")
    if pre + ".shot_cut.weight" in ctx.s:
        return o + conv1x1(ctx, x, pre + ".shot_cut")
    return o + x


def oafilter(ctx, x, pre):
    """oanet.py:56-93 OAFilter on [B, C, K]."""
    o = relu(batch_norm(ctx, instance_norm(x, 1e-3), pre + ".conv1.1"))
    o = conv1x1(ctx, o, pre + ".conv1.3")
    o = np.swapaxes(o, 1, 2)                                   # trans(1,2): [B, K, C]
    o2 = relu(batch_norm(ctx, o, pre + ".conv2.0"))
    o = o + conv1x1(ctx, o2, pre + ".conv2.2")
    o = np.swapaxes(o, 1, 2)                                   # back to [B, C, K]
    o = relu(batch_norm(ctx, instance_norm(o, 1e-3), pre + ".conv3.2"))
    o = conv1x1(ctx, o, pre + ".conv3.4")
    return o + x


def softmax(x, axis):
    m = x.max(axis=axis, keepdims=True)
    e = np.exp(x - m)
    return e / e.sum(axis=axis, keepdims=True)


def diff_pool(ctx, x, pre):
    """oanet.py:96-110: S = softmax_N(conv(x)) [B, K, N]; out = x S^T [B, C, K]."""
    e = conv1x1(ctx, relu(batch_norm(ctx, instance_norm(x, 1e-3), pre + ".conv.1")), pre + ".conv.3")
    S = softmax(e, axis=2)
    return np.matmul(x, np.swapaxes(S, 1, 2))


def diff_unpool(ctx, x_up, x_down, pre):
    """oanet.py:113-129: S = softmax_K(conv(x_up)) [B, K, N]; out = x_down S [B, C, N]."""
    e = conv1x1(ctx, relu(batch_norm(ctx, instance_norm(x_up, 1e-3), pre + ".conv.1")), pre + ".conv.3")
    S = softmax(e, axis=1)
    return np.matmul(x_down, S)


def oanblock(ctx, data, xs, pre, n_layers):
    """oanet.py:165-185.  data [B, Cin, N]; xs [B, N, 6]."""
    x11 = conv1x1(ctx, data, pre + ".conv1")
    for i in range(n_layers // 2):
        x11 = pointcn(ctx, x11, "%s.l1_1.%d" % (pre, i))
    xd = diff_pool(ctx, x11, pre + ".down1")
    for i in range(n_layers // 2):
        xd = oafilter(ctx, xd, "%s.l2.%d" % (pre, i))
    xu = diff_unpool(ctx, x11, xd, pre + ".up1")
    out = np.concatenate([x11, xu], axis=1)
    for i in range(n_layers // 2):
        out = pointcn(ctx, out, "%s.l1_2.%d" % (pre, i))
    logits = conv1x1(ctx, out, pre + ".output")[:, 0, :]                 # :174
    weights = relu(np.tanh(logits))                                       # :175
    if np.any(weights.sum(axis=1) == 0.0):                                # :177-178
        weights = weights + ctx.dt.type(1.0 / weights.shape[1])
    x1, x2 = xs[:, :, :3], xs[:, :, 3:6]                                  # :180
    R, t, res, flag = kabsch(x1, x2, weights)
    return logits, weights, R, t, res, out, flag


def oanet_forward(state, xs, net_depth=12, iter_num=1, train=False, dtype=np.float32):
    """oanet.py:218-265.  xs [B, N, 6|7] (the reference's data['xs'][:, 0]).
    Returns the reference's output dict with numpy arrays."""
    ctx = _Ctx(state, train, np.dtype(dtype))
    xs = np.asarray(xs, dtype=dtype)
    n_layers = net_depth // (iter_num + 1)
    data = np.swapaxes(xs, 1, 2)                                          # [B, 6, N]
    out = {"logits": [], "scores": [], "rot_est": [], "trans_est": []}
    logits, scores, R, t, res, lat, flag = oanblock(ctx, data, xs, "reg_init", n_layers)
    for lst, v in zip(("logits", "scores", "rot_est", "trans_est"), (logits, scores, R, t)):
        out[lst].append(v)
    for i in range(iter_num):
        inp = np.concatenate([data, res[:, None, :], scores[:, None, :]], axis=1)   # :247-248
        logits, scores, R, t, res, lat, f2 = oanblock(ctx, inp, xs, "reg_iter.%d" % i, n_layers)
        flag = flag or f2
        for lst, v in zip(("logits", "scores", "rot_est", "trans_est"), (logits, scores, R, t)):
            out[lst].append(v)
    out["latent features"] = lat
    out["gradient_flag"] = flag
    return out
