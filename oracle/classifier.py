"""ACFF classifier forward, torch-CPU fp32 restatement (TEST INFRASTRUCTURE ONLY).

acff.py:37-59: cat(dw3x3 d1p0, dw3x3 d2p1, dw3x3 d3p2) -> 1x1 conv -> LeakyReLU(0.01)
-> BatchNorm(eval, eps 1e-5) -> Dropout(eval: identity).
squeeze_ernet.py:24-45, squeeze_ernet_redconv.py:27-52, ernet.py:25-49.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def _t(sd, k):
    v = sd[k]
    return v if isinstance(v, torch.Tensor) else torch.as_tensor(v)


def acff(sd, p, x, hook=None):
    """hook(block, concat, fused_w, fused_b) -> (concat, fused_w, fused_b): the int8 scheme
    model (oracle/int8.py) rewrites the 1x1 fusion GEMM's operands."""
    c = x.shape[1]
    b1 = F.conv2d(x, _t(sd, p + ".conv1.weight"), _t(sd, p + ".conv1.bias"), 1, 0, 1, c)
    b2 = F.conv2d(x, _t(sd, p + ".conv2.weight"), _t(sd, p + ".conv2.bias"), 1, 1, 2, c)
    b3 = F.conv2d(x, _t(sd, p + ".conv3.weight"), _t(sd, p + ".conv3.bias"), 1, 2, 3, c)
    out = torch.cat((b1, b2, b3), 1)
    w, b = _t(sd, p + ".fused_conv.weight"), _t(sd, p + ".fused_conv.bias")
    if hook is not None:
        out, w, b = hook(p, out, w, b)
    out = F.conv2d(out, w, b)
    out = F.leaky_relu(out, 0.01)
    out = F.batch_norm(out, _t(sd, p + ".batch_norm.running_mean"), _t(sd, p + ".batch_norm.running_var"),
                       _t(sd, p + ".batch_norm.weight"), _t(sd, p + ".batch_norm.bias"), False, 0.1, 1e-5)
    return out


def forward(kind: str, sd: dict, x: torch.Tensor, hook=None):
    """x: [N,3,S,S] fp32 -> (logits [N,5], probs [N,5], {block: output}); hook: see acff."""
    sd = {k: (v if isinstance(v, torch.Tensor) else torch.as_tensor(v)).float() for k, v in sd.items()}
    blocks = {}
    out = F.conv2d(x, sd["conv1.weight"], None, 2, 0)
    if kind == "squeeze-redconv":
        out = F.conv2d(out, sd["conv_red1.weight"], sd["conv_red1.bias"])
        out = blocks["acff1"] = acff(sd, "acff1", out, hook)
        out = F.max_pool2d(out, 2, 2)
        out = blocks["acff2"] = acff(sd, "acff2", out, hook)
        out = F.conv2d(out, sd["conv_red2.weight"], sd["conv_red2.bias"])
        out = F.max_pool2d(out, 2, 2)
        out = blocks["acff3"] = acff(sd, "acff3", out, hook)
        out = F.max_pool2d(out, 2, 2)
        out = F.conv2d(out, sd["conv_red3.weight"], sd["conv_red3.bias"])
        out = blocks["acff4"] = acff(sd, "acff4", out, hook)
        pool_pad, nf = 1, 20
    elif kind == "squeeze-ernet":
        out = blocks["acff1"] = acff(sd, "acff1", out, hook)
        out = F.max_pool2d(out, 2, 2)
        out = blocks["acff2"] = acff(sd, "acff2", out, hook)
        out = F.max_pool2d(out, 2, 2)
        out = blocks["acff3"] = acff(sd, "acff3", out, hook)
        out = F.max_pool2d(out, 2, 2)
        out = blocks["acff4"] = acff(sd, "acff4", out, hook)
        pool_pad, nf = 1, 20
    elif kind == "ernet":
        for i, pool in ((1, True), (2, True), (3, True), (4, False), (5, False), (6, False)):
            out = blocks[f"acff{i}"] = acff(sd, f"acff{i}", out, hook)
            if pool:
                out = F.max_pool2d(out, 2, 2)
        pool_pad, nf = 0, 45
    else:
        raise ValueError(kind)
    out = F.conv2d(out, sd["conv2.weight"], None)
    out = F.avg_pool2d(out, 5, 1, pool_pad)
    out = out.reshape(-1, nf)
    logits = F.linear(out, sd["fc.weight"], sd["fc.bias"])
    return logits, F.softmax(logits, dim=1), blocks
