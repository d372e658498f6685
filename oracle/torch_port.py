"""The reference's CPU op sequence restated on torch CPU tensors (TEST / BASELINE INFRASTRUCTURE ONLY).

bench.py's cpu_baseline times this port on the GPU box's host cores: it is what the reference's own
PyTorch code does on a CPU (the reference cannot travel to the box), op for op, in its batches:

  soft_nn      <- /root/reference/lib/layers.py:44-88 + lib/utils.py:968-992: the full [B, N, M] distance matrix,
                  softmax over it, and a bmm with the target coordinates (both directions are computed by the
                  reference's PairwiseReg, lib/pairwise/__init__.py:110-111)
  kabsch       <- lib/utils.py:164-237: weight normalisation, weighted means, the N x N diag_embed weight matrix,
                  torch.svd, the det sign fix, residuals (:240-256)
  oanet_forward <- lib/filtering/oanet.py:18-265: PointCN / diff_pool / OAFilter / diff_unpool as 1x1 convs
                  (matmuls), InstanceNorm / BatchNorm (eval: running stats; train: batch stats), the batch-coupled
                  zero-row guard, two blocks.

Its outputs equal oracle/oanet.py's up to fp32 summation order (tests/test_oracle_golden.py checks it); the
arithmetic reference for parity stays the numpy oracle and the golden fixtures."""
import torch


def _p(state, k):
    return torch.as_tensor(state[k], dtype=torch.float32)


def instance_norm(x, eps):
    m = x.mean(dim=2, keepdim=True)
    v = ((x - m) ** 2).mean(dim=2, keepdim=True)
    return (x - m) / torch.sqrt(v + eps)


def batch_norm(state, x, pre, train, eps=1e-5):
    g, b = _p(state, pre + ".weight"), _p(state, pre + ".bias")
    if train:
        m = x.mean(dim=(0, 2), keepdim=True)
        v = ((x - m) ** 2).mean(dim=(0, 2), keepdim=True)
    else:
        m = _p(state, pre + ".running_mean")[None, :, None]
        v = _p(state, pre + ".running_var")[None, :, None]
    return (x - m) / torch.sqrt(v + eps) * g[None, :, None] + b[None, :, None]


def conv1x1(state, x, pre):
    y = torch.matmul(_p(state, pre + ".weight")[:, :, 0, 0], x)
    if pre + ".bias" in state:
        y = y + _p(state, pre + ".bias")[None, :, None]
    return y


def pointcn(state, x, pre, train):
    o = torch.relu(batch_norm(state, instance_norm(x, 1e-5), pre + ".conv.1", train))
    o = conv1x1(state, o, pre + ".conv.3")
    o = torch.relu(batch_norm(state, instance_norm(o, 1e-5), pre + ".conv.5", train))
    o = conv1x1(state, o, pre + ".conv.7")
    if pre + ".shot_cut.weight" in state:
        return o + conv1x1(state, x, pre + ".shot_cut")
    return o + x


def oafilter(state, x, pre, train):
    o = torch.relu(batch_norm(state, instance_norm(x, 1e-3), pre + ".conv1.1", train))
    o = conv1x1(state, o, pre + ".conv1.3").transpose(1, 2)
    o = o + conv1x1(state, torch.relu(batch_norm(state, o, pre + ".conv2.0", train)), pre + ".conv2.2")
    o = o.transpose(1, 2)
    o = torch.relu(batch_norm(state, instance_norm(o, 1e-3), pre + ".conv3.2", train))
    return conv1x1(state, o, pre + ".conv3.4") + x


def kabsch(x1, x2, w, eps=1e-7):
    """lib/utils.py:164-237 with the reference's N x N diag_embed covariance"""
    w = w / (w.sum(dim=1, keepdim=True) + eps)
    wv = w[:, :, None]
    den = wv.sum(dim=1)[:, None, :] + eps
    x1m = torch.bmm(wv.transpose(1, 2), x1) / den
    x2m = torch.bmm(wv.transpose(1, 2), x2) / den
    x1c, x2c = x1 - x1m, x2 - x2m
    cov = torch.bmm(torch.bmm(x1c.transpose(1, 2), torch.diag_embed(w)), x2c)
    u, s, v = torch.svd(cov)
    d = torch.det(torch.bmm(v, u.transpose(1, 2)))
    D = torch.eye(3).repeat(x1.shape[0], 1, 1)
    D[:, 2, 2] = d
    R = torch.bmm(v, torch.bmm(D, u.transpose(1, 2)))
    t = x2m.transpose(1, 2) - torch.bmm(R, x1m.transpose(1, 2))
    res = torch.norm((torch.bmm(R, x1.transpose(1, 2)) + t).transpose(1, 2) - x2, dim=2)
    return R, t, res


def oanblock(state, data, xs, pre, n_layers, train):
    x11 = conv1x1(state, data, pre + ".conv1")
    for i in range(n_layers // 2):
        x11 = pointcn(state, x11, "%s.l1_1.%d" % (pre, i), train)
    e = conv1x1(state, torch.relu(batch_norm(state, instance_norm(x11, 1e-3), pre + ".down1.conv.1", train)),
                pre + ".down1.conv.3")
    xd = torch.matmul(x11, torch.softmax(e, dim=2).transpose(1, 2))
    for i in range(n_layers // 2):
        xd = oafilter(state, xd, "%s.l2.%d" % (pre, i), train)
    e = conv1x1(state, torch.relu(batch_norm(state, instance_norm(x11, 1e-3), pre + ".up1.conv.1", train)),
                pre + ".up1.conv.3")
    out = torch.cat([x11, torch.matmul(xd, torch.softmax(e, dim=1))], dim=1)
    for i in range(n_layers // 2):
        out = pointcn(state, out, "%s.l1_2.%d" % (pre, i), train)
    logits = conv1x1(state, out, pre + ".output")[:, 0, :]
    w = torch.relu(torch.tanh(logits))
    if bool((w.sum(dim=1) == 0).any()):
        w = w + 1.0 / w.shape[1]
    R, t, res = kabsch(xs[:, :, :3], xs[:, :, 3:6], w)
    return logits, w, R, t, res


def oanet_forward(state, xs, net_depth=12, train=False):
    """two blocks (iter_num 1): xs [B, N, 6] float32 torch tensor -> (R, t) of the last block"""
    n_layers = net_depth // 2
    data = xs.transpose(1, 2)
    _, w, R, t, res = oanblock(state, data, xs, "reg_init", n_layers, train)
    inp = torch.cat([data, res[:, None, :], w[:, None, :]], dim=1)
    logits, w, R, t, _ = oanblock(state, inp, xs, "reg_iter.0", n_layers, train)
    return logits, R, t


def soft_nn(x_f, y_f, y_c, temp=0.3, min_temp=1e-4):
    """soft matching, forward value (no straight-through): softmax(-d / tau^2) @ y_c"""
    d = -2.0 * torch.bmm(x_f, y_f.transpose(1, 2))
    d = d + (x_f ** 2).sum(-1)[:, :, None] + (y_f ** 2).sum(-1)[:, None, :]
    tau2 = max(temp * temp, min_temp)
    return torch.bmm(torch.softmax(-d / tau2, dim=2), y_c)
