"""Deterministic synthetic inputs and weights (no network: no datasets, no checkpoints).

* ``synth_frames``: uint8 RGB aerial-like frames [n, h, w, 3] — smooth random
  terrain + random rectangles ("buildings / vehicles") + sensor noise.  Frame i of
  a global batch depends only on (seed, i), so any frame sharding reproduces the
  same global batch.
* ``synth_darknet_weights``: a darknet weight stream (load_darknet_weights order,
  victim_localization/yolov3/models.py:449-486) for a cfg: He-scaled conv
  weights, BN gamma=1/beta=0 with running statistics calibrated once on
  synthetic frames (``data/synth_<cfg>.npz``, produced by
  tests/golden/make_synth.py from the reference model itself) so activations stay
  O(1), and head objectness biases set for a realistic detection rate.
* ``synth_classifier_state_dict``: random-init state dict of the ACFF models.
"""
from __future__ import annotations

import json
import os
import re

import numpy as np

DATA_DIR = os.path.join(os.path.dirname(os.path.abspath(__file__)), "data")
BASE_SEED = 20251015


def synth_frames(n: int, h: int, w: int, seed: int = BASE_SEED, first: int = 0) -> np.ndarray:
    out = np.empty((n, h, w, 3), np.uint8)
    for k in range(n):
        rng = np.random.default_rng(seed + first + k)
        # low-frequency terrain: bilinear upsample of a coarse random grid per channel
        gh, gw = max(2, h // 64), max(2, w // 64)
        coarse = rng.uniform(40, 200, size=(gh, gw, 3)).astype(np.float32)
        ys = np.linspace(0, gh - 1, h, dtype=np.float32)
        xs = np.linspace(0, gw - 1, w, dtype=np.float32)
        y0 = np.floor(ys).astype(int).clip(0, gh - 2)
        x0 = np.floor(xs).astype(int).clip(0, gw - 2)
        fy = (ys - y0)[:, None, None]
        fx = (xs - x0)[None, :, None]
        a = coarse[y0][:, x0]
        b = coarse[y0][:, x0 + 1]
        c = coarse[y0 + 1][:, x0]
        d = coarse[y0 + 1][:, x0 + 1]
        img = (a * (1 - fy) * (1 - fx) + b * (1 - fy) * fx + c * fy * (1 - fx) + d * fy * fx)
        # objects
        for _ in range(int(rng.integers(8, 24))):
            oh, ow = int(rng.integers(6, max(7, h // 8))), int(rng.integers(6, max(7, w // 8)))
            oy, ox = int(rng.integers(0, h - oh)), int(rng.integers(0, w - ow))
            img[oy:oy + oh, ox:ox + ow] = rng.uniform(0, 255, size=3)
        img += rng.normal(0, 6, size=img.shape).astype(np.float32)
        out[k] = np.clip(img, 0, 255).astype(np.uint8)
    return out


# ------------------------------------------------------------------ darknet --
def parse_cfg_text(text: str):
    """parse_model_cfg (yolov3/utils/parse_config.py:6-52) on cfg text."""
    lines = [x for x in text.split("\n") if x and not x.startswith("#")]
    lines = [x.strip() for x in lines]
    mdefs = []
    for line in lines:
        if not line:
            continue
        if line.startswith("["):
            mdefs.append({"type": line[1:-1].rstrip()})
            if mdefs[-1]["type"] == "convolutional":
                mdefs[-1]["batch_normalize"] = 0
        else:
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


def conv_layers(cfg_text: str):
    """[(layer_idx, cin, cout, k, bn, head_no)] in weight-stream order (head_no = nc+5 for a
    conv feeding a [yolo] layer, else 0)."""
    mdefs = parse_cfg_text(cfg_text)
    net = mdefs.pop(0)
    filters_out = [int(net.get("channels", 3))]
    convs = []
    for i, m in enumerate(mdefs):
        t = m["type"]
        if t == "convolutional":
            f = int(m["filters"])
            nxt = mdefs[i + 1] if i + 1 < len(mdefs) else {"type": ""}
            head_no = int(nxt["classes"]) + 5 if nxt["type"] == "yolo" else 0
            convs.append((i, filters_out[-1], f, int(m["size"]), int(m["batch_normalize"]), head_no))
        elif t == "route":
            f = sum(filters_out[l + 1 if l > 0 else l] for l in m["layers"])
        elif t in ("shortcut", "maxpool", "upsample", "yolo"):
            f = filters_out[-1]
        elif t == "acff":
            f = int(m["filters"])
        else:
            raise ValueError(f"unsupported layer type {t}")
        filters_out.append(f)
    return convs


def acff_layers(cfg_text: str):
    """[(layer_idx, cin, cout)] of the [acff] blocks (models.py:46-55 -> ACFF :265-315)."""
    mdefs = parse_cfg_text(cfg_text)
    net = mdefs.pop(0)
    filters_out = [int(net.get("channels", 3))]
    out = []
    for i, m in enumerate(mdefs):
        t = m["type"]
        if t in ("convolutional", "acff"):
            f = int(m["filters"])
            if t == "acff":
                out.append((i, filters_out[-1], f))
        elif t == "route":
            f = sum(filters_out[l + 1 if l > 0 else l] for l in m["layers"])
        else:
            f = filters_out[-1]
        filters_out.append(f)
    return out


ACFF_KEYS = ("conv1.weight", "conv1.bias", "conv2.weight", "conv2.bias", "conv3.weight", "conv3.bias",
             "fused_conv.weight", "fused_conv.bias", "batch_norm.weight", "batch_norm.bias",
             "batch_norm.running_mean", "batch_norm.running_var")


def synth_acff_params(cfg_text: str, seed: int = 9, calib: dict | None = None, preset: str = "he",
                      cond: dict | None = None, conv_seed: int = 7) -> dict:
    """{layer: {ACFF state-dict key: array}} for a Darknet cfg's [acff] blocks.  These are
    not in a .weights stream (load_darknet_weights, models.py:457-486, loads only
    [convolutional]); the reference gets them from a .pt state dict.  Depthwise branches
    He-scaled over their 9 taps and down-weighted by 1/sqrt(3) (three are summed), the 1x1
    He-scaled, BN gamma 1 / beta 0 with running stats from `calib` (acffmean<i>/acffvar<i>).
    preset "cond": the well-conditioned set's blocks (drawn in the same cfg walk as its
    conv stream, seeded by conv_seed / seed)."""
    if preset == "cond":
        return _cond_generate(cfg_text, conv_seed, seed, calib, cond or COND)[1]
    rng = np.random.default_rng(seed)
    out = {}
    for (i, c, f) in acff_layers(cfg_text):
        p = {}
        for b in (1, 2, 3):
            p[f"conv{b}.weight"] = (rng.standard_normal((c, 1, 3, 3), dtype=np.float32)
                                    * np.float32(np.sqrt(2.0 / 9.0 / 3.0)))
            p[f"conv{b}.bias"] = (rng.standard_normal(c, dtype=np.float32) * np.float32(0.05))
        p["fused_conv.weight"] = rng.standard_normal((f, c, 1, 1), dtype=np.float32) * np.float32(np.sqrt(2.0 / c))
        p["fused_conv.bias"] = rng.standard_normal(f, dtype=np.float32) * np.float32(0.05)
        p["batch_norm.weight"] = np.ones(f, np.float32)
        p["batch_norm.bias"] = np.zeros(f, np.float32)
        if calib is not None and f"acffobj{i}" in calib:  # head ACFF: objectness shift
            p["batch_norm.bias"] = calib[f"acffobj{i}"].astype(np.float32)
        has = calib is not None and f"acffmean{i}" in calib
        p["batch_norm.running_mean"] = calib[f"acffmean{i}"].astype(np.float32) if has else np.zeros(f, np.float32)
        p["batch_norm.running_var"] = calib[f"acffvar{i}"].astype(np.float32) if has else np.ones(f, np.float32)
        out[i] = p
    return out


def cfg_name(cfg_path_or_name: str) -> str:
    return re.sub(r"\.cfg$", "", os.path.basename(cfg_path_or_name))


def load_calibration(name: str, preset: str = "he"):
    path = os.path.join(DATA_DIR, f"synth_{name}.npz" if preset == "he" else f"synth_{name}_{preset}.npz")
    if not os.path.exists(path):
        return None
    z = np.load(path, allow_pickle=False)
    return {k: z[k] for k in z.files}


def synth_darknet_weights(cfg_text: str, seed: int = 7, calib: dict | None = None,
                          obj_bias: float = -3.5, preset: str = "he", cond: dict | None = None) -> np.ndarray:
    """Float32 darknet weight stream (after the 20-byte header) for cfg_text.
    preset "he": mean-field He-scaled random convs; "cond": the well-conditioned set
    (see COND below)."""
    if preset == "cond":
        return _cond_generate(cfg_text, seed, 9, calib, cond or COND)[0]
    rng = np.random.default_rng(seed)
    parts = []
    for (i, cin, cout, k, bn, head) in conv_layers(cfg_text):
        fan_in = cin * k * k
        w = rng.standard_normal((cout, cin, k, k), dtype=np.float32) * np.float32(np.sqrt(2.0 / fan_in))
        if bn:
            beta = np.zeros(cout, np.float32)
            gamma = np.ones(cout, np.float32)
            mean = np.zeros(cout, np.float32)
            var = np.ones(cout, np.float32)
            if calib is not None and f"mean{i}" in calib:
                mean = calib[f"mean{i}"].astype(np.float32)
                var = calib[f"var{i}"].astype(np.float32)
            parts += [beta, gamma, mean, var]
        else:
            bias = np.zeros(cout, np.float32)
            if head:
                w *= np.float32(np.sqrt(0.5))  # head: unit-variance logits
                ob = float(calib[f"objbias{i}"]) if calib is not None and f"objbias{i}" in calib else obj_bias
                for a in range(cout // head):
                    bias[a * head + 4] = ob
            parts.append(bias)
        parts.append(w.reshape(-1))
    return np.concatenate(parts).astype(np.float32)


# ------------------------------------------------- well-conditioned weights --
# The "he" set above is mean-field random: every layer is a fresh He-scaled random map
# whose BatchNorm re-centres and re-normalises its output, so a perturbation of an
# activation (an fp16 or int8 rounding) grows ~1.16x per LeakyReLU layer relative to the
# signal (the activation's DC part carries norm that BN removes) -- a 75-conv net turns
# fp16 storage noise into pixel-scale box errors.  Trained detectors are not like that:
# their filters are smooth and their channel maps low-rank.  The "cond" set models that:
#   * each conv's output channels are a rank-r mix (A: cout x r) of r latent maps, and
#     each conv reads its input through the producing layer's basis U (cin x r), so
#     rounding noise spread over all cin channels is projected onto r of them while the
#     signal (which lives in span U) passes: W = A . M . U^T (+ a small full-rank part so
#     every channel and tap still feeds every output, as the fp32 parity bars need);
#   * the r x r x 3 x 3 mixing taps M are mostly a smooth binomial kernel (white rounding
#     noise is averaged, smooth features pass);
#   * a residual branch's last conv writes into the stream's own basis, at BatchNorm
#     gamma `gamma_res`;
#   * head rows are scaled per field by calibration (`headgain<i>`: x,y logits std 1,
#     w,h std 0.25 -- boxes near their anchors, as trained YOLO heads are -- objectness
#     and class logits std 2) and the objectness bias set for ~2 % of anchors at obj > 0.3.
# Only elementwise float64 arithmetic in a fixed order (no BLAS, no reductions), so the
# stream is bit-identical on any host.
COND = {"rank": 16, "iso": 0.05, "lp": 0.85, "gamma_res": 0.5, "obj_pass": 0.002,
        "head_std": {"xy": 1.0, "wh": 0.1, "obj": 2.0, "cls": 2.0}}
_BINOM = np.outer([1.0, 2.0, 1.0], [1.0, 2.0, 1.0]) / 6.0  # unit Frobenius norm


def _gauss(rng, shape, std):
    return rng.standard_normal(shape) * std


def _lowrank_w(rng, U, A, cout, k, cond, stem_hp=None):
    """cout x cin x k x k float64: sqrt(1-iso) * (A M U^T, He-scaled) + sqrt(iso) * He."""
    cin, rin = U.shape
    fan = cin * k * k
    rout = A.shape[1] if A is not None else cout
    g = rng.standard_normal((rout, rin))
    if k == 1:
        M = g[:, :, None, None]
    elif stem_hp is not None:  # the frame-reading stem: random taps, DC part scaled by (1 - stem_hp)
        e = rng.standard_normal((rout, rin, k, k))
        tot = np.zeros(e.shape[:2])
        for t in range(k * k):  # fixed-order sum: no numpy reduction (bit-stable across hosts)
            tot = tot + e[:, :, t // k, t % k]
        M = e - (stem_hp * tot / (k * k))[:, :, None, None]
    else:
        e = rng.standard_normal((rout, rin, k, k)) / float(k)
        M = g[:, :, None, None] * (np.sqrt(cond["lp"]) * _BINOM) + e * np.sqrt(1.0 - cond["lp"])
    T = np.zeros((rout, cin, k, k))
    for l in range(rin):
        T += M[:, l][:, None] * U[None, :, l, None, None]
    if A is None:  # head: outputs read the latents directly
        W = T
        var = rin / cin / (k * k)
    else:
        W = np.zeros((cout, cin, k, k))
        for j in range(rout):
            W += A[:, j, None, None, None] * T[j][None]
        var = rout * rin / cout / cin / (k * k)
    he = 2.0 / fan
    W *= np.sqrt(he * (1.0 - cond["iso"]) / var)
    W += _gauss(rng, (cout, cin, k, k), np.sqrt(he * cond["iso"]))
    return W


def _cond_generate(cfg_text: str, seed: int, acff_seed: int, calib: dict | None, cond: dict):
    """(darknet stream float32, {acff layer: params}) of the well-conditioned set.  A
    calibration file records the knobs it was made with (`cond_json`); they win."""
    if calib is not None and "cond_json" in calib:
        cond = json.loads(str(calib["cond_json"]))
    rng = np.random.default_rng(seed)
    arng = np.random.default_rng(acff_seed)
    mdefs = parse_cfg_text(cfg_text)
    net = mdefs.pop(0)
    c0 = int(net.get("channels", 3))
    fout = [c0]
    basis = [np.eye(c0)]
    r = cond["rank"]
    parts, acff = [], {}

    def new_basis(c):
        return _gauss(rng, (c, min(r, c)), 1.0 / np.sqrt(c))

    def cal(key, default):
        return calib[key] if calib is not None and key in calib else default

    for i, m in enumerate(mdefs):
        t = m["type"]
        nxt = mdefs[i + 1] if i + 1 < len(mdefs) else {"type": ""}
        U = basis[-1]
        if t == "convolutional":
            f, k, bn = int(m["filters"]), int(m["size"]), int(m["batch_normalize"])
            head = nxt["type"] == "yolo"
            A, res = None, False
            if not head:
                if nxt["type"] == "shortcut":
                    fr = nxt["from"][0]
                    src = basis[i + 2 + fr if fr < 0 else fr + 1]
                    res = src.shape[0] == f
                A = src if res else new_basis(f)
            w = _lowrank_w(rng, U, A, f, k, cond, stem_hp=cond.get("stem_hp") if i == 0 else None).astype(np.float32)
            if bn:
                beta = np.zeros(f, np.float32)
                gamma = np.full(f, cond["gamma_res"] if res else 1.0, np.float32)
                parts += [beta, gamma, cal(f"mean{i}", np.zeros(f, np.float32)).astype(np.float32),
                          cal(f"var{i}", np.ones(f, np.float32)).astype(np.float32)]
            else:
                bias = np.zeros(f, np.float32)
                if head:
                    w *= cal(f"headgain{i}", np.ones(f, np.float32)).astype(np.float32)[:, None, None, None]
                    no = int(nxt["classes"]) + 5
                    for a in range(f // no):
                        bias[a * no + 4] = float(cal(f"objbias{i}", -3.5))
                parts.append(bias)
            parts.append(w.reshape(-1))
            basis.append(A if A is not None else new_basis(f))
        elif t == "acff":
            f = int(m["filters"])
            c = U.shape[0]
            p = {}
            for b in (1, 2, 3):  # shared smooth tap + a small per-channel part
                dw = (np.sqrt(cond["lp"]) * _BINOM)[None, None] + _gauss(arng, (c, 1, 3, 3), np.sqrt(1 - cond["lp"]) / 3)
                p[f"conv{b}.weight"] = (dw * np.sqrt(1.0 / 3.0)).astype(np.float32)
                p[f"conv{b}.bias"] = _gauss(arng, c, 0.05).astype(np.float32)
            head = nxt["type"] == "yolo"
            A = None if head else _gauss(arng, (f, min(r, f)), 1.0 / np.sqrt(f))
            p["fused_conv.weight"] = _lowrank_w(arng, U, A, f, 1, cond).astype(np.float32)
            p["fused_conv.bias"] = cal(f"acffbias{i}", _gauss(arng, f, 0.05)).astype(np.float32)
            p["batch_norm.weight"] = cal(f"acffgain{i}", np.ones(f, np.float32)).astype(np.float32)
            p["batch_norm.bias"] = cal(f"acffobj{i}", np.zeros(f, np.float32)).astype(np.float32)
            p["batch_norm.running_mean"] = cal(f"acffmean{i}", np.zeros(f, np.float32)).astype(np.float32)
            p["batch_norm.running_var"] = cal(f"acffvar{i}", np.ones(f, np.float32)).astype(np.float32)
            acff[i] = p
            basis.append(A if A is not None else _gauss(arng, (f, min(r, f)), 1.0 / np.sqrt(f)))
            fout.append(f)
            continue
        elif t == "route":
            ls = [l if l < 0 else l + 1 for l in m["layers"]]  # index into basis/fout (input at 0)
            ls = [len(basis) + l if l < 0 else l for l in ls]
            bs = [basis[l] for l in ls]
            rows = sum(b.shape[0] for b in bs)
            cols = sum(b.shape[1] for b in bs)
            B = np.zeros((rows, cols))
            ro = co = 0
            for b in bs:
                B[ro:ro + b.shape[0], co:co + b.shape[1]] = b
                ro += b.shape[0]
                co += b.shape[1]
            basis.append(B)
            fout.append(rows)
            continue
        elif t in ("shortcut", "maxpool", "upsample", "yolo"):
            basis.append(U)
        else:
            raise ValueError(f"unsupported layer type {t}")
        fout.append(basis[-1].shape[0])
    return np.concatenate(parts).astype(np.float32), acff


def write_darknet_weights(path: str, stream: np.ndarray) -> None:
    """models.py:489-512 format: int32[3] version, int64 seen, float32 stream."""
    with open(path, "wb") as f:
        np.array([0, 2, 5], dtype=np.int32).tofile(f)
        np.array([0], dtype=np.int64).tofile(f)
        np.asarray(stream, np.float32).tofile(f)


def read_darknet_weights(path: str) -> np.ndarray:
    """load_darknet_weights header handling (models.py:449-455)."""
    with open(path, "rb") as f:
        np.fromfile(f, dtype=np.int32, count=3)
        np.fromfile(f, dtype=np.int64, count=1)
        return np.fromfile(f, dtype=np.float32)


# --------------------------------------------------------------- classifier --
def classifier_param_shapes(kind: str):
    """state_dict key -> shape for 'squeeze-ernet' | 'squeeze-redconv' | 'ernet'."""
    shapes = {"conv1.weight": (16, 3, 3, 3)}
    if kind == "squeeze-ernet":
        blocks = [("acff1", 16, 64), ("acff2", 64, 96), ("acff3", 96, 128), ("acff4", 128, 256)]
        fc_in = 20
    elif kind == "squeeze-redconv":
        blocks = [("acff1", 8, 64), ("acff2", 64, 96), ("acff3", 48, 128), ("acff4", 64, 256)]
        shapes.update({"conv_red1.weight": (8, 16, 1, 1), "conv_red1.bias": (8,),
                       "conv_red2.weight": (48, 96, 1, 1), "conv_red2.bias": (48,),
                       "conv_red3.weight": (64, 128, 1, 1), "conv_red3.bias": (64,)})
        fc_in = 20
    elif kind == "ernet":
        blocks = [("acff1", 16, 64), ("acff2", 64, 96), ("acff3", 96, 128), ("acff4", 128, 128),
                  ("acff5", 128, 128), ("acff6", 128, 256)]
        fc_in = 45
    else:
        raise ValueError(f"Unsupported model: {kind}")
    for name, cin, cout in blocks:
        for b in (1, 2, 3):
            shapes[f"{name}.conv{b}.weight"] = (cin, 1, 3, 3)
            shapes[f"{name}.conv{b}.bias"] = (cin,)
        shapes[f"{name}.fused_conv.weight"] = (cout, 3 * cin, 1, 1)
        shapes[f"{name}.fused_conv.bias"] = (cout,)
        for k in ("weight", "bias", "running_mean", "running_var"):
            shapes[f"{name}.batch_norm.{k}"] = (cout,)
    shapes["conv2.weight"] = (5, 256, 1, 1)
    shapes["fc.weight"] = (5, fc_in)
    shapes["fc.bias"] = (5,)
    return shapes


def synth_classifier_state_dict(kind: str, seed: int = 11):
    rng = np.random.default_rng(seed)
    sd = {}
    for k, shp in classifier_param_shapes(kind).items():
        if k.endswith("running_var"):
            v = rng.uniform(0.5, 2.0, size=shp)
        elif k.endswith("running_mean") or k.endswith(".bias"):
            v = rng.normal(0, 0.1, size=shp)
        elif k.endswith("batch_norm.weight"):
            v = rng.uniform(0.8, 1.2, size=shp)
        else:
            fan_in = int(np.prod(shp[1:]))
            v = rng.normal(0, np.sqrt(2.0 / fan_in), size=shp)
        sd[k] = v.astype(np.float32)
    return sd


def acff_stream(params: dict) -> np.ndarray:
    """One [acff] block's parameters in the detector stream order: conv1 w, b, conv2 w, b,
    conv3 w, b, fused_conv w, b, BN gamma, beta, running mean, running var."""
    return np.concatenate([np.asarray(params[k], np.float32).reshape(-1) for k in ACFF_KEYS])


def inline_acff(cfg_text: str, conv_stream: np.ndarray, acff: dict) -> np.ndarray:
    """Darknet conv stream (models.py:457-486 order) with each [acff] block's parameters
    inserted at its layer position: the stream rtdm_detector_create takes for YOLO-ACFF."""
    if not acff:
        return conv_stream
    parts, ptr = [], 0
    convs = {i: (cin, cout, k, bn) for (i, cin, cout, k, bn, _) in conv_layers(cfg_text)}
    for i in sorted(set(convs) | set(acff)):
        if i in acff:
            parts.append(acff_stream(acff[i]))
        else:
            cin, cout, k, bn = convs[i]
            n = (4 * cout if bn else cout) + cout * cin * k * k
            parts.append(conv_stream[ptr:ptr + n])
            ptr += n
    assert ptr == conv_stream.size, (ptr, conv_stream.size)
    return np.concatenate(parts).astype(np.float32)

