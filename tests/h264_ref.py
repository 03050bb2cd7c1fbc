"""Independent Python references for the H.264 inter decoder tests (tests/test_h264_inter.py):
the in-loop deblocking filter (H.264 8.7), luma / chroma motion compensation (8.4.2.2) and
motion-vector prediction (8.4.1.3), written from the standard's equations - they share no code
with ``arbius_amd/native/src/h264.cpp``."""
from __future__ import annotations

import numpy as np

ALPHA = [0] * 16 + [4, 4, 5, 6, 7, 8, 9, 10, 12, 13, 15, 17, 20, 22, 25, 28, 32, 36, 40, 45, 50, 56, 63, 71, 80, 90,
                    101, 113, 127, 144, 162, 182, 203, 226, 255, 255]
BETA = [0] * 16 + [2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13, 14, 14, 15,
                   15, 16, 16, 17, 17, 18, 18]
TC0 = [[0, 0, 0]] * 17 + [[0, 0, 1]] * 4 + [[0, 1, 1]] * 2 + [[1, 1, 1]] * 4 + [[1, 1, 2]] * 4 + [
    [1, 2, 3], [1, 2, 3], [2, 2, 3], [2, 2, 4], [2, 3, 4], [2, 3, 4], [3, 3, 5], [3, 4, 6], [3, 4, 6], [4, 5, 7],
    [4, 5, 8], [4, 6, 9], [5, 7, 10], [6, 8, 11], [6, 8, 13], [7, 10, 14], [8, 11, 16], [9, 12, 18], [10, 13, 20],
    [11, 15, 23], [13, 17, 25]]
QPC = list(range(30)) + [29, 30, 31, 32, 32, 33, 34, 34, 35, 35, 36, 36, 37, 37, 37, 38, 38, 38, 39, 39, 39, 39]
assert len(ALPHA) == len(BETA) == len(TC0) == len(QPC) == 52


def clip3(lo, hi, v):
    return lo if v < lo else hi if v > hi else v


def _filter_line(s, bS, chroma, alpha, beta, idx_a):
    """s: list of 8 samples p3 p2 p1 p0 q0 q1 q2 q3 (chroma: only p1 p0 q0 q1 used) -> filtered list."""
    p3, p2, p1, p0, q0, q1, q2, q3 = s
    if not (abs(p0 - q0) < alpha and abs(p1 - p0) < beta and abs(q1 - q0) < beta):
        return s
    out = list(s)
    ap, aq = abs(p2 - p0), abs(q2 - q0)
    if bS < 4:
        tc0 = TC0[idx_a][bS - 1]
        tc = tc0 + 1 if chroma else tc0 + (ap < beta) + (aq < beta)
        delta = clip3(-tc, tc, (((q0 - p0) << 2) + (p1 - q1) + 4) >> 3)
        out[3] = clip3(0, 255, p0 + delta)
        out[4] = clip3(0, 255, q0 - delta)
        if not chroma and ap < beta:
            out[2] = p1 + clip3(-tc0, tc0, (p2 + ((p0 + q0 + 1) >> 1) - (p1 << 1)) >> 1)
        if not chroma and aq < beta:
            out[5] = q1 + clip3(-tc0, tc0, (q2 + ((p0 + q0 + 1) >> 1) - (q1 << 1)) >> 1)
        return out
    if not chroma and ap < beta and abs(p0 - q0) < ((alpha >> 2) + 2):
        out[3] = (p2 + 2 * p1 + 2 * p0 + 2 * q0 + q1 + 4) >> 3
        out[2] = (p2 + p1 + p0 + q0 + 2) >> 2
        out[1] = (2 * p3 + 3 * p2 + p1 + p0 + q0 + 4) >> 3
    else:
        out[3] = (2 * p1 + p0 + q1 + 2) >> 2
    if not chroma and aq < beta and abs(p0 - q0) < ((alpha >> 2) + 2):
        out[4] = (p1 + 2 * p0 + 2 * q0 + 2 * q1 + q2 + 4) >> 3
        out[5] = (p0 + q0 + q1 + q2 + 2) >> 2
        out[6] = (2 * q3 + 3 * q2 + q1 + q0 + p0 + 4) >> 3
    else:
        out[4] = (2 * q1 + q0 + p1 + 2) >> 2
    return out


def deblock(side, W, H):
    """Apply the deblocking filter to side['y'/'cb'/'cr'] (unfiltered) with the per-block inputs the
    decoder recorded; returns filtered (Y, Cb, Cr) as int arrays."""
    mbw, mbh = W // 16, H // 16
    Y = side["y"].astype(np.int64).reshape(H, W).copy()
    planes = [side["cb"].astype(np.int64).reshape(H // 2, W // 2).copy(),
              side["cr"].astype(np.int64).reshape(H // 2, W // 2).copy()]
    bw4 = 4 * mbw
    mvx, mvy = side["mvx"].reshape(-1), side["mvy"].reshape(-1)
    refpic, nz = side["refpic"].reshape(-1), side["nonzero"].reshape(-1)
    intra, qp, slc = side["intra"], side["qp"].astype(int), side["slice"]
    cqo = side["chroma_qp_offset"]

    def bs(p, q, mb_edge):                     # p, q: (bx, by) absolute 4x4 luma block coordinates
        pm, qm = (p[1] // 4) * mbw + p[0] // 4, (q[1] // 4) * mbw + q[0] // 4
        if intra[pm] or intra[qm]:
            return 4 if mb_edge else 3
        pi, qi = p[1] * bw4 + p[0], q[1] * bw4 + q[0]
        if nz[pi] or nz[qi]:
            return 2
        if refpic[pi] != refpic[qi] or abs(int(mvx[pi]) - int(mvx[qi])) >= 4 or abs(int(mvy[pi]) - int(mvy[qi])) >= 4:
            return 1
        return 0

    for mb in range(mbw * mbh):
        mx, my = mb % mbw, mb // mbw
        idc, offa, offb = side["deblock"][slc[mb]]
        if idc == 1:
            continue
        for vertical in (True, False):
            for e in range(4):
                if e == 0:
                    nmb = mb - 1 if vertical else mb - mbw
                    if (mx == 0 if vertical else my == 0):
                        continue
                    if idc == 2 and slc[nmb] != slc[mb]:
                        continue
                else:
                    nmb = mb
                strengths = []
                for k in range(4):
                    q = (4 * mx + e, 4 * my + k) if vertical else (4 * mx + k, 4 * my + e)
                    p = (q[0] - 1, q[1]) if vertical else (q[0], q[1] - 1)
                    strengths.append(bs(p, q, e == 0))
                # luma
                qpav = (qp[nmb] + qp[mb] + 1) >> 1
                ia, ib = clip3(0, 51, qpav + offa), clip3(0, 51, qpav + offb)
                for k in range(16):
                    b = strengths[k // 4]
                    if b == 0:
                        continue
                    if vertical:
                        y0, x0 = 16 * my + k, 16 * mx + 4 * e
                        line = [int(Y[y0, x0 + d]) for d in range(-4, 4)]
                        new = _filter_line(line, b, False, ALPHA[ia], BETA[ib], ia)
                        for d in range(-4, 4):
                            Y[y0, x0 + d] = new[d + 4]
                    else:
                        y0, x0 = 16 * my + 4 * e, 16 * mx + k
                        line = [int(Y[y0 + d, x0]) for d in range(-4, 4)]
                        new = _filter_line(line, b, False, ALPHA[ia], BETA[ib], ia)
                        for d in range(-4, 4):
                            Y[y0 + d, x0] = new[d + 4]
                if e % 2:
                    continue
                # chroma (4:2:0: the luma edges 0 and 2 are chroma edges 0 and 4)
                qpc = (QPC[clip3(0, 51, qp[nmb] + cqo)] + QPC[clip3(0, 51, qp[mb] + cqo)] + 1) >> 1
                ca, cb_ = clip3(0, 51, qpc + offa), clip3(0, 51, qpc + offb)
                for C in planes:
                    for k in range(8):
                        b = strengths[k // 2]
                        if b == 0:
                            continue
                        if vertical:
                            y0, x0 = 8 * my + k, 8 * mx + 2 * e
                            line = [0, 0] + [int(C[y0, x0 + d]) for d in range(-2, 2)] + [0, 0]
                        else:
                            y0, x0 = 8 * my + 2 * e, 8 * mx + k
                            line = [0, 0] + [int(C[y0 + d, x0]) for d in range(-2, 2)] + [0, 0]
                        new = _filter_line(line, b, True, ALPHA[ca], BETA[cb_], ca)
                        for d in range(-2, 2):
                            if vertical:
                                C[y0, x0 + d] = new[d + 4]
                            else:
                                C[y0 + d, x0] = new[d + 4]
    return Y, planes[0], planes[1]


# ------------------------------------------------------------------------ motion compensation
def _tap(v):
    return v[0] - 5 * v[1] + 20 * v[2] + 20 * v[3] - 5 * v[4] + v[5]


def luma_sample(ref, xq, yq):
    """Quarter-sample luma value at (xq / 4, yq / 4) of reference plane `ref` (8.4.2.2.1), edge-clamped."""
    H, W = ref.shape

    def G(x, y):
        return int(ref[clip3(0, H - 1, y), clip3(0, W - 1, x)])

    def b1(x, y):            # intermediate horizontal half sample between (x, y) and (x + 1, y)
        return _tap([G(x + d, y) for d in range(-2, 4)])

    def h1(x, y):
        return _tap([G(x, y + d) for d in range(-2, 4)])

    def c8(v):
        return clip3(0, 255, v)

    xi, yi, xf, yf = xq >> 2, yq >> 2, xq & 3, yq & 3
    Gv = G(xi, yi)
    b = c8((b1(xi, yi) + 16) >> 5)
    h = c8((h1(xi, yi) + 16) >> 5)
    j = c8((_tap([b1(xi, yi + d) for d in range(-2, 4)]) + 512) >> 10)
    s = c8((b1(xi, yi + 1) + 16) >> 5)         # half sample below b
    m = c8((h1(xi + 1, yi) + 16) >> 5)         # half sample right of h
    avg = lambda u, v: (u + v + 1) >> 1
    table = {
        (0, 0): Gv, (1, 0): avg(Gv, b), (2, 0): b, (3, 0): avg(b, G(xi + 1, yi)),
        (0, 1): avg(Gv, h), (1, 1): avg(b, h), (2, 1): avg(b, j), (3, 1): avg(b, m),
        (0, 2): h, (1, 2): avg(h, j), (2, 2): j, (3, 2): avg(j, m),
        (0, 3): avg(h, G(xi, yi + 1)), (1, 3): avg(h, s), (2, 3): avg(j, s), (3, 3): avg(s, m),
    }
    return table[(xf, yf)]


def chroma_sample(ref, xe, ye):
    """Eighth-sample chroma value at (xe / 8, ye / 8) (8.4.2.2.2), edge-clamped."""
    H, W = ref.shape
    P = lambda x, y: int(ref[clip3(0, H - 1, y), clip3(0, W - 1, x)])
    xi, yi, xf, yf = xe >> 3, ye >> 3, xe & 7, ye & 7
    return ((8 - xf) * (8 - yf) * P(xi, yi) + xf * (8 - yf) * P(xi + 1, yi) + (8 - xf) * yf * P(xi, yi + 1)
            + xf * yf * P(xi + 1, yi + 1) + 32) >> 6


def predict_block(refs, x0, y0, w, h, mv):
    """(Y block, Cb block, Cr block) of a w x h luma partition at (x0, y0) with quarter-sample mv."""
    ry, rcb, rcr = refs
    Yb = np.array([[luma_sample(ry, 4 * (x0 + i) + mv[0], 4 * (y0 + j) + mv[1]) for i in range(w)] for j in range(h)])
    cbs = [np.array([[chroma_sample(c, 8 * (x0 // 2 + i) + mv[0], 8 * (y0 // 2 + j) + mv[1]) for i in range(w // 2)]
                     for j in range(h // 2)]) for c in (rcb, rcr)]
    return Yb, cbs[0], cbs[1]


# ------------------------------------------------------------------------ motion vector prediction
def median(a, b, c):
    return max(min(a, b), min(max(a, b), c))


class MotionField:
    """Per-4x4 motion of one picture (one slice): (ref_idx, mvx, mvy) or None (not available /
    not yet decoded); intra blocks are ('intra')."""

    def __init__(self, mbw, mbh):
        self.mbw, self.mbh = mbw, mbh
        self.blk = {}

    def get(self, bx, by, cur_mb, decoded_in_mb):
        """Neighbour (bx, by) in absolute 4x4 units seen from macroblock cur_mb."""
        if bx < 0 or by < 0 or bx >= 4 * self.mbw or by >= 4 * self.mbh:
            return None
        nb_mb = (by // 4) * self.mbw + bx // 4
        if nb_mb == cur_mb:
            return self.blk.get((bx, by)) if (bx, by) in decoded_in_mb else None
        if nb_mb > cur_mb:
            return None
        return self.blk.get((bx, by))

    def predict(self, mb, x, y, w, h, ref, decoded, shape=None):
        """mvp for the partition at absolute 4x4 (x, y) of size w x h (4x4 units)."""
        A = self.get(x - 1, y, mb, decoded)
        B = self.get(x, y - 1, mb, decoded)
        C = self.get(x + w, y - 1, mb, decoded)
        if C is None:
            C = self.get(x - 1, y - 1, mb, decoded)
        def ref_of(n):
            return -1 if n is None or n == "intra" else n[0]
        def mv_of(n):
            return (0, 0) if n is None or n == "intra" else (n[1], n[2])
        if shape == "16x8_top" and ref_of(B) == ref:
            return mv_of(B)
        if shape == "16x8_bottom" and ref_of(A) == ref:
            return mv_of(A)
        if shape == "8x16_left" and ref_of(A) == ref:
            return mv_of(A)
        if shape == "8x16_right" and ref_of(C) == ref:
            return mv_of(C)
        if B is None and C is None and A is not None:
            B = C = A
        same = [n for n in (A, B, C) if ref_of(n) == ref]
        if len(same) == 1:
            return mv_of(same[0])
        return (median(mv_of(A)[0], mv_of(B)[0], mv_of(C)[0]), median(mv_of(A)[1], mv_of(B)[1], mv_of(C)[1]))

    def skip_mv(self, mb):
        mx, my = mb % self.mbw, mb // self.mbw
        A = self.get(4 * mx - 1, 4 * my, mb, set())
        B = self.get(4 * mx, 4 * my - 1, mb, set())
        if A is None or B is None:
            return (0, 0)
        for n in (A, B):
            if n != "intra" and n[0] == 0 and n[1] == 0 and n[2] == 0:
                return (0, 0)
        return self.predict(mb, 4 * mx, 4 * my, 4, 4, 0, set())

    def set(self, x, y, w, h, val, decoded):
        for j in range(y, y + h):
            for i in range(x, x + w):
                self.blk[(i, j)] = val
                decoded.add((i, j))
