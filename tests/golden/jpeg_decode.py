"""Baseline JPEG decoder with selectable reconstruction arithmetic
(fixture tooling for tests/golden/make_golden.py; TEST INFRASTRUCTURE ONLY).

Why: the reference's golden snapshots were computed from JPEGs decoded by
the `image` crate 0.25.2, whose JPEG backend is zune-jpeg (not in
/root/reference).  JPEG decoders agree on the entropy-decoded coefficients
but differ in the integer arithmetic of three reconstruction steps, and a
+-1 LSB input difference moves SIFT keypoints by ~1e-2 px.  This decoder
does the exact part once (marker parsing, Huffman decoding, dequantisation:
ITU-T T.81) and offers the published variants of the three steps:

  idct      "islow"  libjpeg jidctint.c (13-bit constants, PASS1_BITS 2)
            "stb"    stb_image stbi__idct_block (12-bit constants), which
                     zune-jpeg's integer IDCT follows
  upsample  "libjpeg" h2v2 fancy upsampling (jdsample.c: +8 / +7 rounding)
            "stb"     stbi__resample_row_hv_2 (one combined triangle filter)
            "twopass" vertical then horizontal 3:1 triangle filter, each
                      rounded ((3a + b + 2) >> 2)
  color     "libjpeg" jdcolor.c 16-bit fixed-point tables
            "stb"     stbi__YCbCr_to_RGB_row (20-bit fixed point)
            "zune"    6-bit fixed-point coefficients 45/32, 11/32, 23/32,
                      113/64 in i16 arithmetic
  edge      "clamp"  chroma edge samples replicate the component's real
                     (ceil) size; "pad": use the decoded block padding

`decode(path, idct="islow", upsample="libjpeg", color="libjpeg")` reproduces
libjpeg-turbo (PIL) bit-exactly on the reference images (checked in
make_golden.py); the snapshot-matching combination is recorded there.
Supports baseline sequential Huffman JPEGs (SOF0/SOF1), 1 or 3 components,
any sampling factors of 1 or 2, restart intervals.
"""
import numpy as np

ZIGZAG = np.array([
    0, 1, 8, 16, 9, 2, 3, 10, 17, 24, 32, 25, 18, 11, 4, 5, 12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6, 7, 14, 21,
    28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61,
    54, 47, 55, 62, 63], dtype=np.int64)


# ---------------------------------------------------------------------------
# entropy decoding (exact, ITU-T T.81 F.2)
# ---------------------------------------------------------------------------
class _Bits:
    def __init__(self, data, pos):
        self.d, self.p, self.acc, self.n = data, pos, 0, 0

    def _fill(self):
        while self.n <= 24:
            b = 0
            if self.p < len(self.d):
                b = self.d[self.p]
                if b == 0xFF:
                    nxt = self.d[self.p + 1] if self.p + 1 < len(self.d) else 0
                    if nxt == 0x00:
                        self.p += 2
                    else:  # marker: feed zeros, do not advance
                        b = 0
                else:
                    self.p += 1
            self.acc = (self.acc << 8) | b
            self.n += 8

    def bits(self, k):
        if k == 0:
            return 0
        self._fill()
        self.n -= k
        return (self.acc >> self.n) & ((1 << k) - 1)

    def bit(self):
        return self.bits(1)

    def restart(self):
        # drop buffered bits, skip the RSTn marker
        self.acc, self.n = 0, 0
        while self.p + 1 < len(self.d) and not (self.d[self.p] == 0xFF and 0xD0 <= self.d[self.p + 1] <= 0xD7):
            self.p += 1
        self.p += 2


def _huff_table(counts, symbols):
    """(maxcode, valptr, mincode, symbols) per code length 1..16."""
    code, k = 0, 0
    maxcode, valptr, mincode = [-1] * 17, [0] * 17, [0] * 17
    for ln in range(1, 17):
        if counts[ln - 1]:
            valptr[ln] = k
            mincode[ln] = code
            code += counts[ln - 1]
            k += counts[ln - 1]
            maxcode[ln] = code - 1
        code <<= 1
    return maxcode, valptr, mincode, symbols


def _decode_sym(bs, t):
    maxcode, valptr, mincode, symbols = t
    code = bs.bit()
    for ln in range(1, 17):
        if code <= maxcode[ln]:
            return symbols[valptr[ln] + code - mincode[ln]]
        code = (code << 1) | bs.bit()
    raise ValueError("bad Huffman code")


def _extend(v, t):
    return v - (1 << t) + 1 if t and v < (1 << (t - 1)) else v


def parse(path):
    d = open(path, "rb").read()
    assert d[0] == 0xFF and d[1] == 0xD8
    p = 2
    qt, ht, comps, restart = {}, {}, [], 0
    frame = None
    while p < len(d):
        assert d[p] == 0xFF, "marker expected"
        m = d[p + 1]
        p += 2
        if m == 0xD9:
            break
        ln = (d[p] << 8) | d[p + 1]
        seg = d[p + 2:p + ln]
        if m == 0xDB:  # DQT
            i = 0
            while i < len(seg):
                pq, tq = seg[i] >> 4, seg[i] & 15
                i += 1
                if pq:
                    vals = [(seg[i + 2 * k] << 8) | seg[i + 2 * k + 1] for k in range(64)]
                    i += 128
                else:
                    vals = list(seg[i:i + 64])
                    i += 64
                q = np.zeros(64, np.int64)
                q[ZIGZAG] = vals  # natural order
                qt[tq] = q
        elif m == 0xC4:  # DHT
            i = 0
            while i < len(seg):
                tc, th = seg[i] >> 4, seg[i] & 15
                counts = list(seg[i + 1:i + 17])
                nsym = sum(counts)
                syms = list(seg[i + 17:i + 17 + nsym])
                ht[(tc, th)] = _huff_table(counts, syms)
                i += 17 + nsym
        elif m in (0xC0, 0xC1):  # baseline / extended sequential Huffman
            h, w, nc = (seg[1] << 8) | seg[2], (seg[3] << 8) | seg[4], seg[5]
            for k in range(nc):
                cid, hv, tq = seg[6 + 3 * k], seg[7 + 3 * k], seg[8 + 3 * k]
                comps.append({"id": cid, "h": hv >> 4, "v": hv & 15, "tq": tq})
            frame = (w, h)
        elif m in (0xC2, 0xC3, 0xC5, 0xC6, 0xC7, 0xC9, 0xCA, 0xCB, 0xCD, 0xCE, 0xCF):
            raise NotImplementedError("only baseline sequential Huffman JPEG")
        elif m == 0xDD:
            restart = (seg[0] << 8) | seg[1]
        elif m == 0xDA:  # SOS
            ns = seg[0]
            sel = {}
            for k in range(ns):
                sel[seg[1 + 2 * k]] = (seg[2 + 2 * k] >> 4, seg[2 + 2 * k] & 15)
            for c in comps:
                c["td"], c["ta"] = sel[c["id"]]
            coefs, p = _scan(d, p + ln, frame, comps, qt, ht, restart)
            return frame, comps, coefs
        p += ln
    raise ValueError("no scan")


def _scan(d, p, frame, comps, qt, ht, restart):
    w, h = frame
    hmax, vmax = max(c["h"] for c in comps), max(c["v"] for c in comps)
    mcux, mcuy = -(-w // (8 * hmax)), -(-h // (8 * vmax))
    coefs = [np.zeros((mcuy * c["v"], mcux * c["h"], 64), np.int64) for c in comps]
    bs = _Bits(d, p)
    pred = [0] * len(comps)
    n = 0
    for my in range(mcuy):
        for mx in range(mcux):
            if restart and n and n % restart == 0:
                bs.restart()
                pred = [0] * len(comps)
            n += 1
            for ci, c in enumerate(comps):
                dc_t, ac_t, q = ht[(0, c["td"])], ht[(1, c["ta"])], qt[c["tq"]]
                for by in range(c["v"]):
                    for bx in range(c["h"]):
                        blk = np.zeros(64, np.int64)
                        t = _decode_sym(bs, dc_t)
                        pred[ci] += _extend(bs.bits(t), t)
                        blk[0] = pred[ci]
                        k = 1
                        while k < 64:
                            rs = _decode_sym(bs, ac_t)
                            r, s = rs >> 4, rs & 15
                            if s == 0:
                                if r != 15:
                                    break
                                k += 16
                                continue
                            k += r
                            blk[ZIGZAG[k]] = _extend(bs.bits(s), s)
                            k += 1
                        coefs[ci][my * c["v"] + by, mx * c["h"] + bx] = blk * q  # dequantised, natural order
    return coefs, bs.p


# ---------------------------------------------------------------------------
# IDCT variants (vectorised over blocks; int64 == the C int arithmetic here)
# ---------------------------------------------------------------------------
def _idct_islow(c):
    """libjpeg jidctint.c jpeg_idct_islow (CONST_BITS 13, PASS1_BITS 2)."""
    CB, P1 = 13, 2
    F = {k: v for k, v in dict(f0298=2446, f0390=3196, f0541=4433, f0765=6270, f0899=7373, f1175=9633,
                                   f1501=12299, f1847=15137, f1961=16069, f2053=16819, f2562=20995,
                                   f3072=25172).items()}
    blk = c.reshape(-1, 8, 8)  # [n][row v][col u] natural order: index = v*8 + u

    def one_d(s, shift_even):
        s0, s1, s2, s3, s4, s5, s6, s7 = [s[..., i] for i in range(8)]
        z1 = (s2 + s6) * F["f0541"]
        tmp2 = z1 + s6 * (-F["f1847"])
        tmp3 = z1 + s2 * F["f0765"]
        tmp0 = (s0 + s4) << CB
        tmp1 = (s0 - s4) << CB
        t10, t13, t11, t12 = tmp0 + tmp3, tmp0 - tmp3, tmp1 + tmp2, tmp1 - tmp2
        o0, o1, o2, o3 = s7, s5, s3, s1
        z1, z2, z3, z4 = o0 + o3, o1 + o2, o0 + o2, o1 + o3
        z5 = (z3 + z4) * F["f1175"]
        o0, o1, o2, o3 = o0 * F["f0298"], o1 * F["f2053"], o2 * F["f3072"], o3 * F["f1501"]
        z1, z2, z3, z4 = z1 * (-F["f0899"]), z2 * (-F["f2562"]), z3 * (-F["f1961"]), z4 * (-F["f0390"])
        z3 += z5
        z4 += z5
        o0 += z1 + z3
        o1 += z2 + z4
        o2 += z2 + z3
        o3 += z1 + z4
        return [t10 + o3, t11 + o2, t12 + o1, t13 + o0, t13 - o0, t12 - o1, t11 - o2, t10 - o3]

    def descale(x, n):
        return (x + (1 << (n - 1))) >> n

    # pass 1: columns (s_k = coefficient row k of column u)
    cols = np.transpose(blk, (0, 2, 1))  # [n][u][v]
    ac_zero = np.all(cols[..., 1:] == 0, axis=-1)
    outs = one_d(cols, True)
    ws = np.stack([descale(o, CB - P1) for o in outs], axis=-1)  # [n][u][y]
    ws = np.where(ac_zero[..., None], cols[..., :1] << P1, ws)
    # pass 2: rows (s_k = workspace column k of row y)
    rows = np.transpose(ws, (0, 2, 1))  # [n][y][u]
    outs = one_d(rows, True)
    px = np.stack([descale(o, CB + P1 + 3) for o in outs], axis=-1)  # [n][y][x]
    # libjpeg skips pass-2 work for all-zero AC rows: identical value
    rz = np.all(rows[..., 1:] == 0, axis=-1)
    dc = descale(rows[..., :1], P1 + 3)
    px = np.where(rz[..., None], dc, px)
    return np.clip((px & 1023) + 128 if False else px + 128, 0, 255).reshape(c.shape[:-1] + (8, 8))


def _idct_stb(c, row_bias=65536 + (128 << 17)):
    """stb_image stbi__idct_block (12-bit fixed point).  `row_bias` is the
    rounding + level-shift term of the row pass."""
    def f2f(x):
        return int(x * 4096 + 0.5)

    def one_d(s):
        s0, s1, s2, s3, s4, s5, s6, s7 = [s[..., i] for i in range(8)]
        p2, p3 = s2, s6
        p1 = (p2 + p3) * f2f(0.5411961)
        t2 = p1 + p3 * f2f(-1.847759065)
        t3 = p1 + p2 * f2f(0.765366865)
        p2, p3 = s0, s4
        t0 = (p2 + p3) * 4096
        t1 = (p2 - p3) * 4096
        x0, x3, x1, x2 = t0 + t3, t0 - t3, t1 + t2, t1 - t2
        t0, t1, t2, t3 = s7, s5, s3, s1
        p3, p4, p1, p2 = t0 + t2, t1 + t3, t0 + t3, t1 + t2
        p5 = (p3 + p4) * f2f(1.175875602)
        t0, t1, t2, t3 = t0 * f2f(0.298631336), t1 * f2f(2.053119869), t2 * f2f(3.072711026), t3 * f2f(1.501321110)
        p1 = p5 + p1 * f2f(-0.899976223)
        p2 = p5 + p2 * f2f(-2.562915447)
        p3 = p3 * f2f(-1.961570560)
        p4 = p4 * f2f(-0.390180644)
        t3 += p1 + p4
        t2 += p2 + p3
        t1 += p2 + p4
        t0 += p1 + p3
        return x0, x1, x2, x3, t0, t1, t2, t3

    blk = c.reshape(-1, 8, 8)
    cols = np.transpose(blk, (0, 2, 1))  # [n][u][v]
    x0, x1, x2, x3, t0, t1, t2, t3 = one_d(cols)
    x0, x1, x2, x3 = x0 + 512, x1 + 512, x2 + 512, x3 + 512
    v = np.stack([(x0 + t3) >> 10, (x1 + t2) >> 10, (x2 + t1) >> 10, (x3 + t0) >> 10,
                  (x3 - t0) >> 10, (x2 - t1) >> 10, (x1 - t2) >> 10, (x0 - t3) >> 10], axis=-1)
    ac_zero = np.all(cols[..., 1:] == 0, axis=-1)
    v = np.where(ac_zero[..., None], cols[..., :1] * 4, v)  # [n][u][y]
    rows = np.transpose(v, (0, 2, 1))  # [n][y][u]
    x0, x1, x2, x3, t0, t1, t2, t3 = one_d(rows)
    x0, x1, x2, x3 = x0 + row_bias, x1 + row_bias, x2 + row_bias, x3 + row_bias
    o = np.stack([(x0 + t3) >> 17, (x1 + t2) >> 17, (x2 + t1) >> 17, (x3 + t0) >> 17,
                  (x3 - t0) >> 17, (x2 - t1) >> 17, (x1 - t2) >> 17, (x0 - t3) >> 17], axis=-1)
    return np.clip(o, 0, 255).reshape(c.shape[:-1] + (8, 8))


def _idct_zune(c, row_bias=512 + 65536 + (128 << 17)):
    """zune-jpeg's integer IDCT: stb_image's arithmetic with the row-pass
    bias 512 + 65536 + (128 << 17) (the column pass's 512 carried into the
    row pass), plus a whole-block shortcut: a block whose 63 AC coefficients
    are zero becomes (DC >> 3) + 128 (no rounding term)."""
    out = _idct_stb(c, row_bias)
    flat = c.reshape(-1, 64)
    dc_only = np.all(flat[:, 1:] == 0, axis=1).reshape(c.shape[:-1])
    dcv = np.clip((c[..., 0] >> 3) + 128, 0, 255)
    return np.where(dc_only[..., None, None], dcv[..., None, None], out)


def _planes(coefs, idct):
    f = {"islow": _idct_islow, "stb": _idct_stb, "zune": _idct_zune,
         "zune_b0": lambda c: _idct_zune(c, 65536 + (128 << 17)),
         "stb_b512": lambda c: _idct_stb(c, 512 + 65536 + (128 << 17))}[idct]
    out = []
    for c in coefs:
        by, bx = c.shape[:2]
        px = f(c)  # [by][bx][8][8]
        out.append(np.transpose(px, (0, 2, 1, 3)).reshape(by * 8, bx * 8))
    return out


# ---------------------------------------------------------------------------
# chroma upsampling (h2v2 / h2v1) and colour conversion
# ---------------------------------------------------------------------------
def _up_h(x, mode):
    """2x horizontal triangle filter of rows x[..., w] -> [..., 2w]."""
    left = np.concatenate([x[..., :1], x[..., :-1]], axis=-1)
    right = np.concatenate([x[..., 1:], x[..., -1:]], axis=-1)
    if mode == "twopass":
        e = (3 * x + left + 2) >> 2
        o = (3 * x + right + 2) >> 2
    else:
        raise ValueError(mode)
    out = np.empty(x.shape[:-1] + (2 * x.shape[-1],), np.int64)
    out[..., 0::2], out[..., 1::2] = e, o
    return out


def _up_hv(x, mode):
    """h2v2 upsample of a (h, w) plane to (2h, 2w)."""
    up = np.concatenate([x[:1], x[:-1]], axis=0)
    dn = np.concatenate([x[1:], x[-1:]], axis=0)
    if mode == "twopass":
        top = (3 * x + up + 2) >> 2
        bot = (3 * x + dn + 2) >> 2
        v = np.empty((2 * x.shape[0], x.shape[1]), np.int64)
        v[0::2], v[1::2] = top, bot
        return _up_h(v, "twopass")
    # column sums of the two contributing rows
    cs_top = 3 * x + up
    cs_bot = 3 * x + dn
    out = np.empty((2 * x.shape[0], 2 * x.shape[1]), np.int64)
    for r0, cs in ((0, cs_top), (1, cs_bot)):
        last = np.concatenate([cs[:, :1], cs[:, :-1]], axis=1)
        nxt = np.concatenate([cs[:, 1:], cs[:, -1:]], axis=1)
        if mode == "libjpeg":
            e = (3 * cs + last + 8) >> 4
            o = (3 * cs + nxt + 7) >> 4
            e[:, 0] = (cs[:, 0] * 4 + 8) >> 4
            o[:, -1] = (cs[:, -1] * 4 + 7) >> 4
        elif mode == "stb":
            e = (3 * cs + last + 8) >> 4
            o = (3 * cs + nxt + 8) >> 4
            e[:, 0] = (cs[:, 0] + 2) >> 2
            o[:, -1] = (cs[:, -1] + 2) >> 2
        else:
            raise ValueError(mode)
        out[r0::2, 0::2], out[r0::2, 1::2] = e, o
    return out


def _color(y, cb, cr, mode):
    if mode == "libjpeg":
        S, half = 16, 1 << 15

        def fix(v):
            return int(v * (1 << S) + 0.5)
        x_cr, x_cb = cr - 128, cb - 128
        r = y + ((fix(1.40200) * x_cr + half) >> S)
        b = y + ((fix(1.77200) * x_cb + half) >> S)
        g = y + ((-fix(0.34414) * x_cb + half - fix(0.71414) * x_cr) >> S)
    elif mode == "stb":
        def f2f(v):
            return int(v * 4096.0 + 0.5) << 8
        yf = (y << 20) + (1 << 19)
        x_cr, x_cb = cr - 128, cb - 128
        r = (yf + x_cr * f2f(1.40200)) >> 20
        g = (yf + x_cr * -f2f(0.71414) + ((x_cb * -f2f(0.34414)) & ~0xFFFF)) >> 20
        b = (yf + x_cb * f2f(1.77200)) >> 20
    elif mode == "zune":
        x_cr, x_cb = cr - 128, cb - 128
        r = y + ((45 * x_cr) >> 5)
        g = y - ((11 * x_cb + 23 * x_cr) >> 5)
        b = y + ((113 * x_cb) >> 6)
    else:
        raise ValueError(mode)
    return [np.clip(c, 0, 255) for c in (r, g, b)]


def decode(path, idct="islow", upsample="libjpeg", color="libjpeg", edge="clamp"):
    """(h, w, 3) uint8 RGB (or (h, w) for grayscale JPEGs)."""
    (w, h), comps, coefs = parse(path)
    planes = _planes(coefs, idct)
    if len(comps) == 1:
        return planes[0][:h, :w].astype(np.uint8)
    hmax, vmax = max(c["h"] for c in comps), max(c["v"] for c in comps)
    full = []
    for c, p in zip(comps, planes):
        fh, fv = hmax // c["h"], vmax // c["v"]
        if edge == "clamp":  # the component's real size (ceil), as libjpeg sizes it
            p = p[:-(-h * c["v"] // vmax), :-(-w * c["h"] // hmax)]
        if (fh, fv) == (1, 1):
            q = p
        elif (fh, fv) == (2, 2):
            q = _up_hv(p, upsample)
        elif (fh, fv) == (2, 1):
            q = _up_h(p, "twopass") if upsample == "twopass" else _up_hv_h_only(p, upsample)
        else:
            raise NotImplementedError("sampling factors")
        full.append(q[:h, :w])
    r, g, b = _color(full[0], full[1], full[2], color)
    return np.stack([r, g, b], axis=-1).astype(np.uint8)


def _up_hv_h_only(x, mode):
    """h2v1 fancy upsampling (libjpeg h2v1_fancy_upsample / stb hv... h-only)."""
    last = np.concatenate([x[:, :1], x[:, :-1]], axis=1)
    nxt = np.concatenate([x[:, 1:], x[:, -1:]], axis=1)
    e = (3 * x + last + 1) >> 2
    o = (3 * x + nxt + 2) >> 2
    out = np.empty((x.shape[0], 2 * x.shape[1]), np.int64)
    out[:, 0::2], out[:, 1::2] = e, o
    out[:, 0] = x[:, 0]
    out[:, -1] = x[:, -1]
    return out


def luma(rgb):
    """image 0.25 `grayscale()`: (2126 R + 7152 G + 722 B) / 10000, integer division."""
    rgb = rgb.astype(np.int64)
    return np.clip((2126 * rgb[..., 0] + 7152 * rgb[..., 1] + 722 * rgb[..., 2]) // 10000, 0, 255).astype(np.uint8)
