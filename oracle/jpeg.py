"""Baseline JPEG decode restated in Python / numpy (TEST INFRASTRUCTURE ONLY).

What cv2.imread does to a JPEG in the reference (victim_localization/yolov3/utils/
datasets.py:97, disaster_detection/aider-predict.py:57): libjpeg-turbo's default
decompression.  cv2 is absent from this image; Pillow links the same libjpeg-turbo with
the same defaults (JDCT_ISLOW, do_fancy_upsampling), so Pillow's decode is the reference
output, and this restatement is pinned against it (tests/test_jpeg.py) on the reference's
bundled JPEGs and on Pillow-encoded variants (4:4:4, 4:2:2, restart markers, optimised
Huffman tables, grayscale).  Stages, each after its published algorithm:
  entropy_decode  ITU-T T.81 Annex B markers, Annex C canonical Huffman codes, F.2.2
                  sequential decode (DC prediction, AC run / size), restart intervals;
                  libjpeg's guard for runs past 63 (jpeg_natural_order's extra entries)
  idct_islow      libjpeg jidctint.c (CONST_BITS 13, PASS1_BITS 2, the post-IDCT
                  range-limit table indexed & 1023)
  upsample        libjpeg-turbo jdsample.c h2v2 / h2v1 fancy upsampling (triangle filter,
                  biases 8/7 and 1/2, first / last column cases, edge-replicated context
                  rows; box replication when the downsampled width is <= 2)
  ycc_to_rgb      jdcolor.c ycc_rgb_convert (16-bit fixed point tables)
Pure-Python Huffman decoding: fine for the small test images, slow for large ones.
"""
from __future__ import annotations

import numpy as np

ZIGZAG = np.array([0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13,
                   6, 7, 14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45,
                   38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63] + [63] * 16)


def _huff(counts, vals):
    """{(length, code): symbol} of a canonical table (T.81 C.2)."""
    table, code, k = {}, 0, 0
    for ln in range(1, 17):
        for _ in range(counts[ln - 1]):
            table[(ln, code)] = vals[k]
            code += 1
            k += 1
        code <<= 1
    return table


class _Bits:
    def __init__(self, data, pos):
        self.d, self.p, self.acc, self.n, self.marker = data, pos, 0, 0, False

    def _byte(self):
        if self.marker or self.p >= len(self.d):
            return 0
        b = self.d[self.p]
        if b == 0xFF:
            nxt = self.d[self.p + 1] if self.p + 1 < len(self.d) else 0xD9
            if nxt == 0:
                self.p += 2
                return 0xFF
            self.marker = True
            return 0
        self.p += 1
        return b

    def bit(self):
        if self.n == 0:
            self.acc, self.n = self._byte(), 8
        self.n -= 1
        return (self.acc >> self.n) & 1

    def bits(self, k):
        v = 0
        for _ in range(k):
            v = (v << 1) | self.bit()
        return v

    def decode(self, table):
        code = 0
        for ln in range(1, 17):
            code = (code << 1) | self.bit()
            s = table.get((ln, code))
            if s is not None:
                return s
        return 0  # corrupt: libjpeg returns symbol 0

    def restart(self):
        self.acc = self.n = 0
        d = self.d
        while self.p + 1 < len(d) and not (d[self.p] == 0xFF and 0xD0 <= d[self.p + 1] <= 0xD7):
            self.p += 1
        if self.p + 1 < len(d):
            self.p += 2
        self.marker = False


def _extend(v, s):
    return v - (1 << s) + 1 if v < (1 << (s - 1)) else v


def entropy_decode(data: bytes):
    """-> dict(width, height, comps=[dict(h, v, q[64] natural, coef [bh, bw, 64] int32)])."""
    d = memoryview(data).tobytes()
    assert d[:2] == b"\xff\xd8", "no SOI"
    p, q, dc, ac, ri = 2, {}, {}, {}, 0
    frame = None
    while p < len(d):
        if d[p] != 0xFF:
            p += 1
            continue
        while p < len(d) and d[p] == 0xFF:
            p += 1
        m = d[p]
        p += 1
        if m == 0xD9:
            break
        if m == 0x01 or 0xD0 <= m <= 0xD7:
            continue
        ln = (d[p] << 8) | d[p + 1]
        seg = d[p + 2:p + ln]
        if m in (0xC0, 0xC1):
            h, w, nc = (seg[1] << 8) | seg[2], (seg[3] << 8) | seg[4], seg[5]
            comps = [dict(id=seg[6 + 3 * i], h=seg[7 + 3 * i] >> 4, v=seg[7 + 3 * i] & 15, tq=seg[8 + 3 * i] & 3)
                     for i in range(nc)]
            if nc == 1:
                comps[0]["h"] = comps[0]["v"] = 1
            hmax, vmax = max(c["h"] for c in comps), max(c["v"] for c in comps)
            mcux, mcuy = -(-w // (8 * hmax)), -(-h // (8 * vmax))
            for c in comps:
                c["coef"] = np.zeros((mcuy * c["v"], mcux * c["h"], 64), np.int32)
                c["cbw"] = -(-(-(-w * c["h"] // hmax)) // 8)
                c["cbh"] = -(-(-(-h * c["v"] // vmax)) // 8)
            frame = dict(width=w, height=h, comps=comps, mcux=mcux, mcuy=mcuy)
        elif 0xC2 <= m <= 0xCF and m not in (0xC4, 0xC8, 0xCC):
            raise NotImplementedError("only sequential Huffman JPEGs")
        elif m == 0xDB:
            i = 0
            while i < len(seg):
                pq, t = seg[i] >> 4, seg[i] & 3
                i += 1
                tab = np.zeros(64, np.int32)
                for k in range(64):
                    if pq:
                        tab[ZIGZAG[k]] = (seg[i] << 8) | seg[i + 1]
                        i += 2
                    else:
                        tab[ZIGZAG[k]] = seg[i]
                        i += 1
                q[t] = tab
        elif m == 0xC4:
            i = 0
            while i < len(seg):
                tc, th = seg[i] >> 4, seg[i] & 3
                counts = list(seg[i + 1:i + 17])
                vals = list(seg[i + 17:i + 17 + sum(counts)])
                (ac if tc else dc)[th] = _huff(counts, vals)
                i += 17 + sum(counts)
        elif m == 0xDD:
            ri = (seg[0] << 8) | seg[1]
        elif m == 0xDA:
            ns = seg[0]
            sc = []
            for k in range(ns):
                cid, t = seg[1 + 2 * k], seg[2 + 2 * k]
                c = next(c for c in frame["comps"] if c["id"] == cid)
                c["td"], c["ta"] = t >> 4, t & 3
                sc.append(c)
            p = _scan(frame, sc, dc, ac, ri, d, p + ln)
            continue
        p += ln
    for c in frame["comps"]:
        c["q"] = q[c["tq"]]
    return frame


def _scan(frame, sc, dc, ac, ri, d, pos):
    b = _Bits(d, pos)
    pred = {id(c): 0 for c in sc}
    inter = len(sc) > 1
    if inter:
        mcus, cols = frame["mcux"] * frame["mcuy"], frame["mcux"]
    else:
        mcus, cols = sc[0]["cbw"] * sc[0]["cbh"], sc[0]["cbw"]

    def block(c, by, bx):
        blk = c["coef"][by, bx]
        blk[:] = 0
        t = b.decode(dc[c["td"]])
        if t:
            pred[id(c)] += _extend(b.bits(t), t)
        v = pred[id(c)] & 0xFFFF  # the JCOEF (short) store
        blk[0] = v - 0x10000 if v >= 0x8000 else v
        k = 1
        while k < 64:
            rs = b.decode(ac[c["ta"]])
            r, s = rs >> 4, rs & 15
            if s:
                k += r
                blk[ZIGZAG[k]] = _extend(b.bits(s), s)
            else:
                if r != 15:
                    break
                k += 15
            k += 1

    todo = ri
    for mi in range(mcus):
        if ri:
            if todo == 0:
                b.restart()
                for key in pred:
                    pred[key] = 0
                todo = ri
            todo -= 1
        my, mx = divmod(mi, cols)
        if inter:
            for c in sc:
                for v in range(c["v"]):
                    for h in range(c["h"]):
                        block(c, my * c["v"] + v, mx * c["h"] + h)
        else:
            block(sc[0], my, mx)
    p = b.p
    while p + 1 < len(d) and not (d[p] == 0xFF and d[p + 1] != 0 and not 0xD0 <= d[p + 1] <= 0xD7):
        p += 1
    return p


C = dict(F0_298=2446, F0_390=3196, F0_541=4433, F0_765=6270, F0_899=7373, F1_175=9633, F1_501=12299, F1_847=15137,
         F1_961=16069, F2_053=16819, F2_562=20995, F3_072=25172)


def _idct1(z, n):
    """jidctint.c's 8-point pass over axis -1 of int64 z (..., 8) -> descaled by n bits."""
    z0, z1, z2, z3, z4, z5, z6, z7 = (z[..., i] for i in range(8))
    zz = (z2 + z6) * C["F0_541"]
    tmp2 = zz + z6 * -C["F1_847"]
    tmp3 = zz + z2 * C["F0_765"]
    t0, t1 = (z0 + z4) << 13, (z0 - z4) << 13
    tmp10, tmp13, tmp11, tmp12 = t0 + tmp3, t0 - tmp3, t1 + tmp2, t1 - tmp2
    a0, a1, a2, a3 = z7, z5, z3, z1
    q1, q2, q3, q4 = a0 + a3, a1 + a2, a0 + a2, a1 + a3
    z5_ = (q3 + q4) * C["F1_175"]
    a0, a1, a2, a3 = a0 * C["F0_298"], a1 * C["F2_053"], a2 * C["F3_072"], a3 * C["F1_501"]
    q1, q2, q3, q4 = q1 * -C["F0_899"], q2 * -C["F2_562"], q3 * -C["F1_961"] + z5_, q4 * -C["F0_390"] + z5_
    a0, a1, a2, a3 = a0 + q1 + q3, a1 + q2 + q4, a2 + q2 + q3, a3 + q1 + q4
    r = 1 << (n - 1)
    out = [tmp10 + a3, tmp11 + a2, tmp12 + a1, tmp13 + a0, tmp13 - a0, tmp12 - a1, tmp11 - a2, tmp10 - a3]
    return np.stack([(o + r) >> n for o in out], -1)


def _range_limit(x):
    v = x & 1023
    return np.where(v < 128, v + 128, np.where(v < 512, 255, np.where(v < 896, 0, v - 896))).astype(np.uint8)


def idct_islow(coef, q):
    """coef [..., 64] natural order, q [64] -> samples [..., 8, 8] uint8."""
    x = coef.astype(np.int64) * q.astype(np.int64)
    x = x.reshape(x.shape[:-1] + (8, 8))
    ws = _idct1(np.swapaxes(x, -1, -2), 13 - 2)           # columns: [..., col, row]
    out = _idct1(np.swapaxes(ws, -1, -2), 13 + 2 + 3)     # rows
    return _range_limit(out)


def plane(c):
    """A component's sample plane [bh*8, bw*8] from its coefficient grid."""
    s = idct_islow(c["coef"], c["q"])                      # [bh, bw, 8, 8]
    bh, bw = s.shape[:2]
    return s.transpose(0, 2, 1, 3).reshape(bh * 8, bw * 8)


def upsample(pl, cw, ch, hf, vf, out_w, out_h):
    """libjpeg-turbo fancy upsampling of the valid cw x ch part of pl to out_w x out_h."""
    s = pl[:ch, :cw].astype(np.int32)
    if hf == 1 and vf == 1:
        return s[:out_h, :out_w]
    xs = np.arange(out_w)
    cx = xs >> 1
    if vf == 1:  # h2v1
        if cw <= 2:
            return s[:out_h, cx]
        left = s[:, np.maximum(cx - 1, 0)]
        right = s[:, np.minimum(cx + 1, cw - 1)]
        me = s[:, cx]
        even = np.where(cx == 0, me, (me * 3 + left + 1) >> 2)
        odd = np.where(cx == cw - 1, me, (me * 3 + right + 2) >> 2)
        return np.where((xs & 1) == 0, even, odd)[:out_h]
    ys = np.arange(out_h)
    cy = ys >> 1
    if cw <= 2:
        return s[cy][:, cx]
    ny = np.where(ys & 1, np.minimum(cy + 1, ch - 1), np.maximum(cy - 1, 0))
    colsum = s[cy] * 3 + s[ny]                            # [out_h, cw]
    th = colsum[:, cx]
    lt = colsum[:, np.maximum(cx - 1, 0)]
    rt = colsum[:, np.minimum(cx + 1, cw - 1)]
    even = np.where(cx == 0, (th * 4 + 8) >> 4, (th * 3 + lt + 8) >> 4)
    odd = np.where(cx == cw - 1, (th * 4 + 7) >> 4, (th * 3 + rt + 7) >> 4)
    return np.where((xs & 1) == 0, even, odd)


def ycc_to_rgb(y, cb, cr):
    cb, cr = cb.astype(np.int64) - 128, cr.astype(np.int64) - 128
    y = y.astype(np.int64)
    r = y + ((91881 * cr + 32768) >> 16)
    g = y + ((-22554 * cb + 32768 - 46802 * cr) >> 16)
    b = y + ((116130 * cb + 32768) >> 16)
    return np.clip(np.stack([r, g, b], -1), 0, 255).astype(np.uint8)


def decode(data: bytes) -> np.ndarray:
    """JPEG bytes -> uint8 [H, W, 3] RGB (grayscale replicated, as cv2.imread's colour mode)."""
    f = entropy_decode(data)
    w, h, comps = f["width"], f["height"], f["comps"]
    y = plane(comps[0])[:h, :w]
    if len(comps) == 1:
        return np.repeat(y[..., None], 3, -1).astype(np.uint8)
    hmax = max(c["h"] for c in comps)
    vmax = max(c["v"] for c in comps)
    hf, vf = comps[0]["h"], comps[0]["v"]
    cw, ch = -(-w * comps[1]["h"] // hmax), -(-h * comps[1]["v"] // vmax)
    cb = upsample(plane(comps[1]), cw, ch, hf, vf, w, h)
    cr = upsample(plane(comps[2]), cw, ch, hf, vf, w, h)
    return ycc_to_rgb(y, cb, cr)


def coefficients(data: bytes):
    """[nblocks, 64] int16 in rtdm_jpeg_entropy_decode's layout (components in order, each
    grid row-major) + the quant tables [ncomp, 64]."""
    f = entropy_decode(data)
    blocks = np.concatenate([c["coef"].reshape(-1, 64) for c in f["comps"]])
    return blocks.astype(np.int16), np.stack([c["q"] for c in f["comps"]]).astype(np.uint16)
