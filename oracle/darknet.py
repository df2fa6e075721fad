"""Darknet forward + YOLO decode, torch-CPU fp32 restatement (TEST INFRASTRUCTURE ONLY).

Restates yolov3/utils/parse_config.py:6-52 (cfg parse), models.py:9-123
(create_modules: conv(bias=!bn) + BN(eps 1e-4) + LeakyReLU(0.1)/Swish; maxpool
with ZeroPad2d for size 2 / stride 1; nearest upsample; route concat; shortcut
add), models.py:449-486 (weight stream order), models.py:332-395 (forward) and
models.py:204-258 + 422-436 (YOLOLayer inference decode, create_grids), and the
[acff] block (models.py:46-55 -> ACFF.forward :296-315: three dilated depthwise 3x3
branches d1p0 / d2p1 / d3p2 with bias, ADDED, then 1x1 conv + bias, LeakyReLU(0.01),
BatchNorm2d(eps 1e-5, eval), Dropout(eval) -- its parameters come from a state dict, not
the .weights stream).
"""
from __future__ import annotations

import numpy as np
import torch
import torch.nn.functional as F


def parse_cfg(text: str):
    lines = [x for x in text.split("\n") if x and not x.startswith("#")]
    lines = [x.rstrip().lstrip() for x in lines]
    mdefs = []
    for line in lines:
        if line.startswith("["):
            mdefs.append({"type": line[1:-1].rstrip()})
            if mdefs[-1]["type"] == "convolutional":
                mdefs[-1]["batch_normalize"] = 0
        elif line:
            key, val = line.split("=")
            key = key.rstrip()
            if key == "anchors":
                mdefs[-1][key] = np.array([float(x) for x in val.split(",")]).reshape((-1, 2))
            elif key in ("from", "layers", "mask"):
                mdefs[-1][key] = [int(x) for x in val.split(",")]
            else:
                val = val.strip()
                if val.isnumeric():
                    mdefs[-1][key] = int(val) if (int(val) - float(val)) == 0 else float(val)
                else:
                    mdefs[-1][key] = val
    return mdefs


class DarknetRef:
    def __init__(self, cfg_text: str, stream: np.ndarray, acff: dict | None = None):
        """acff: {layer index: {ACFF state-dict key (conv1.weight, ...): array}}."""
        self.mdefs = parse_cfg(cfg_text)
        self.net = self.mdefs.pop(0)
        self.params = {}
        ptr = 0
        cin = [int(self.net.get("channels", 3))]
        self.routs = set()
        for i, m in enumerate(self.mdefs):
            t = m["type"]
            if t == "convolutional":
                f, k = int(m["filters"]), int(m["size"])
                p = {}
                if m["batch_normalize"]:
                    for name in ("beta", "gamma", "mean", "var"):
                        p[name] = torch.from_numpy(stream[ptr:ptr + f].copy())
                        ptr += f
                else:
                    p["bias"] = torch.from_numpy(stream[ptr:ptr + f].copy())
                    ptr += f
                nw = f * cin[-1] * k * k
                p["w"] = torch.from_numpy(stream[ptr:ptr + nw].copy()).view(f, cin[-1], k, k)
                ptr += nw
                self.params[i] = p
            elif t == "acff":
                f = int(m["filters"])
                assert acff is not None and i in acff, f"[acff] layer {i} needs its parameters"
                self.params[i] = {k: torch.from_numpy(np.asarray(v, np.float32).copy()) for k, v in acff[i].items()}
            elif t == "route":
                f = sum(cin[l + 1 if l > 0 else l] for l in m["layers"])
                self.routs.update(i + l if l < 0 else l for l in m["layers"])
            elif t == "shortcut":
                f = cin[-1]
                self.routs.update(i + l if l < 0 else l for l in m["from"])
            else:
                f = cin[-1]
            cin.append(f)
        assert ptr == stream.size, (ptr, stream.size)

    @torch.no_grad()
    def forward(self, x: torch.Tensor, keep_layers=False, raw=False, f16_storage=False, conv_hook=None,
                override=None):
        """x: [N,3,H,W] fp32 in [0,1] -> io [N, sum(A*ny*nx), 5+nc] (and per-layer outputs).
        raw=True: the undecoded p rows instead (YOLOLayer training branch, models.py:240-250).

        f16_storage=True: NOT the reference -- a model of what an fp16 inference engine
        does to it (the reference's own --half path, detect.py:58-60, stores every
        activation in fp16 too): BN folded into the conv weights (eps 1e-4), weights and the
        input rounded to fp16, fp32 arithmetic, every layer output rounded to fp16 except the
        raw head maps (decoded in fp32).  The fp16 parity tests bound the HIP fp16 io's
        deviation from the fp32 oracle by a small multiple of this mode's own deviation.

        conv_hook(i, x, w, b) -> (x, w, b): test-only hook on each [convolutional] layer's
        input and BN-folded weights (f16_storage mode), e.g. to model int8 quantisation.

        override {layer: tensor}: teacher forcing -- after layer i is computed (kept in
        self.computed[i]), later layers consume override[i] instead (e.g. the HIP path's own
        output of that layer), so each layer's deviation is its own, not compounded."""
        h16 = (lambda t: t.half().float()) if f16_storage else (lambda t: t)
        self.computed = {}
        img_size = x.shape[-2:]
        x = h16(x)
        out, io_list = [], []
        self.heads = []  # per [yolo]: grid and masked anchors (the TRT plugin's fields)
        for i, m in enumerate(self.mdefs):
            t = m["type"]
            if t == "convolutional":
                p = self.params[i]
                k = int(m["size"])
                s = int(m["stride"])
                pad = (k - 1) // 2 if m["pad"] else 0
                if f16_storage:
                    w, b = p["w"].double(), p.get("bias")
                    if "gamma" in p:
                        sc = p["gamma"].double() / torch.sqrt(p["var"].double() + 1e-4)
                        w = w * sc.view(-1, 1, 1, 1)
                        b = (p["beta"].double() - p["mean"].double() * sc).float()
                    w = h16(w.float())
                    if conv_hook is not None:
                        x, w, b = conv_hook(i, x, w, b)
                    x = F.conv2d(x, w, b, s, pad)
                else:
                    x = F.conv2d(x, p["w"], p.get("bias"), s, pad)
                    if "gamma" in p:
                        x = F.batch_norm(x, p["mean"], p["var"], p["gamma"], p["beta"], False, 0.003, 1e-4)
                if m["activation"] == "leaky":
                    x = F.leaky_relu(x, 0.1)
                elif m["activation"] == "swish":
                    x = x * torch.sigmoid(x)
            elif t == "acff":
                p = self.params[i]
                c = x.shape[1]
                y = (F.conv2d(x, p["conv1.weight"], p["conv1.bias"], 1, 0, 1, c)
                     + F.conv2d(x, p["conv2.weight"], p["conv2.bias"], 1, 1, 2, c)
                     + F.conv2d(x, p["conv3.weight"], p["conv3.bias"], 1, 2, 3, c))
                y = F.leaky_relu(F.conv2d(h16(y), h16(p["fused_conv.weight"]), p["fused_conv.bias"]), 0.01)
                x = F.batch_norm(y, p["batch_norm.running_mean"], p["batch_norm.running_var"],
                                 p["batch_norm.weight"], p["batch_norm.bias"], False, 0.1, 1e-5)
            elif t == "maxpool":
                k, s = int(m["size"]), int(m["stride"])
                if k == 2 and s == 1:
                    x = F.max_pool2d(F.pad(x, (0, 1, 0, 1)), k, s, (k - 1) // 2)
                else:
                    x = F.max_pool2d(x, k, s, (k - 1) // 2)
            elif t == "upsample":
                x = F.interpolate(x, scale_factor=int(m["stride"]), mode="nearest")
            elif t == "route":
                ls = m["layers"]
                if len(ls) == 1:
                    x = out[ls[0]]
                else:
                    ws = [out[l].shape[-1] for l in ls]
                    if len(ls) == 2 and ws[0] != ws[1]:
                        # models.py:364-375: on a size mismatch the narrower of the two maps
                        # is nearest-resized to the wider one's width, in place in `out`
                        big = 0 if (ws[0], 0) > (ws[1], 1) else 1
                        small = ls[1 - big]
                        out[small] = F.interpolate(out[small], size=max(ws))
                    x = torch.cat([out[l] for l in ls], 1)
            elif t == "shortcut":
                # weightedFeatureFusion.forward (models.py:135-155), unweighted
                a = out[m["from"][0]]
                nc, ac = x.shape[1], a.shape[1]
                if nc > ac:
                    x = x.clone()
                    x[:, :ac] = x[:, :ac] + a
                elif nc < ac:
                    x = x + a[:, :nc]
                else:
                    x = x + a
            elif t == "yolo":
                self.heads.append({"na": len(m["mask"]), "ny": x.shape[2], "nx": x.shape[3],
                                   "anchors": [tuple(m["anchors"][a]) for a in m["mask"]],
                                   "scale_x_y": float(m.get("scale_x_y", 1.0)),
                                   "new_coords": int(m.get("new_coords", 0))})
                io_list.append(self._raw(m, x) if raw else self._yolo(m, x, img_size))
            else:
                raise ValueError(t)
            nxt = self.mdefs[i + 1]["type"] if i + 1 < len(self.mdefs) else ""
            if t != "yolo" and nxt != "yolo":
                x = h16(x)
            if override is not None:
                self.computed[i] = x
                if i in override:
                    x = override[i].to(x.dtype)
            out.append(x if (keep_layers or i in self.routs or override is not None) else [])
        io = torch.cat(io_list, 1)
        return (io, out) if keep_layers else io

    @staticmethod
    def _raw(m, p):
        na, no = len(m["mask"]), int(m["classes"]) + 5
        bs, _, ny, nx = p.shape
        return p.view(bs, na, no, ny, nx).permute(0, 1, 3, 4, 2).reshape(bs, -1, no)

    @staticmethod
    def _yolo(m, p, img_size):
        anchors = torch.Tensor(m["anchors"][m["mask"]])
        na, nc = len(m["mask"]), int(m["classes"])
        no = nc + 5
        bs, _, ny, nx = p.shape
        isz = max(img_size)
        stride = isz / max((nx, ny))
        yv, xv = torch.meshgrid([torch.arange(ny), torch.arange(nx)], indexing="ij")
        grid_xy = torch.stack((xv, yv), 2).float().view((1, 1, ny, nx, 2))
        anchor_wh = (anchors / stride).view(1, na, 1, 1, 2)
        p = p.view(bs, na, no, ny, nx).permute(0, 1, 3, 4, 2).contiguous()
        io = p.clone()
        io[..., :2] = torch.sigmoid(io[..., :2]) + grid_xy
        io[..., 2:4] = torch.exp(io[..., 2:4]) * anchor_wh
        io[..., :4] *= stride
        torch.sigmoid_(io[..., 4:])
        return io.view(bs, -1, no)
