#!/usr/bin/env python3
"""Where the GPU intra encoder's workspace first differs from the host run of the same code
(ops/csrc/h264_intra.hip): per picture, the first macroblock whose info / levels / bit offset /
reconstruction / TotalCoeff differ, for each diagonal hand-off mode (arb_set_h264_sync 0 / 1).
(The round-6 per-optimisation-level runs in profiles/r6/h264/dbg_O*.log also dumped one macroblock's
chroma predictor state through a hook of the earlier one-lane kernel, since removed.)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests"))


def split(ws, F, H16, W16):
    import numpy as np
    mbw, mbh = W16 // 16, H16 // 16
    nmb = mbw * mbh
    sizes = [("lv", nmb * 768), ("info", nmb * 4), ("bits", nmb * 4), ("ry", H16 * W16), ("rcb", H16 * W16 // 4),
             ("rcr", H16 * W16 // 4), ("tcy", 16 * nmb), ("tccb", 4 * nmb), ("tccr", 4 * nmb)]
    per = (sum(n for _, n in sizes) + 255) // 256 * 256
    out = []
    for f in range(F):
        b = ws[f * per:(f + 1) * per]
        d, o = {}, 0
        for k, n in sizes:
            d[k] = b[o:o + n]
            o += n
        d["lv"] = d["lv"].view(np.int16).reshape(nmb, 384)
        d["info"] = d["info"].view(np.uint32)
        d["bits"] = d["bits"].view(np.uint32)
        d["ry"] = d["ry"].reshape(H16, W16)
        out.append(d)
    return out


def main():
    import numpy as np
    import torch

    from arbius_amd.ops import _lib
    from test_h264_gpu_algo import planes
    dev = torch.device("cuda", 0)
    for kind, F, H16, W16, qp in [("smooth", 2, 32, 48, 20), ("noise", 3, 64, 80, 20), ("smooth", 1, 144, 176, 20)]:
        y, cb, cr = planes(kind, F, H16, W16, F * H16 + W16 + qp)
        _, hm, hws = _lib.h264_intra_host(y, cb, cr, qp, return_ws=True)
        H = split(hws, F, H16, W16)
        for mode in (0, 1):
            _lib.lib().arb_set_h264_sync(mode)
            _, gm, gws = _lib.h264_intra_encode(*[torch.from_numpy(p).to(dev) for p in (y, cb, cr)], qp, return_ws=True)
            G = split(gws.cpu().numpy(), F, H16, W16)
            gm = gm.cpu().numpy()
            rep = {"case": [kind, F, H16, W16], "sync": mode, "meta_equal": bool((gm == hm).all())}
            mbw = W16 // 16
            for f in range(F):
                first = {}
                for k in ("info", "bits", "lv"):
                    bad = np.nonzero((G[f][k] != H[f][k]).reshape(len(G[f][k]), -1).any(axis=1))[0]
                    if len(bad):
                        first[k] = [int(bad[0]) % mbw, int(bad[0]) // mbw, len(bad)]
                bad = np.argwhere(G[f]["ry"] != H[f]["ry"])
                if len(bad):
                    first["ry"] = [int(bad[0][1]) // 16, int(bad[0][0]) // 16, len(bad)]
                for k in ("rcb", "rcr", "tcy", "tccb", "tccr"):
                    n = int((G[f][k] != H[f][k]).sum())
                    if n:
                        first[k] = n
                rep[f"pic{f}"] = first or "equal"
                if "info" in first:           # the first differing macroblock, decoded
                    mx, my = first["info"][:2]
                    mb = my * mbw + mx

                    def dec(v):
                        v = int(v)
                        return dict(mode=v & 3, cmode=(v >> 2) & 3, cbpc=(v >> 4) & 3, cbpl=(v >> 6) & 1)
                    cy0, cx0, Wc = 8 * my, 8 * mx, W16 // 2
                    det = {"mb": [mx, my], "host": dec(H[f]["info"][mb]), "gpu": dec(G[f]["info"][mb])}
                    for k in ("rcb", "rcr"):
                        for name, D in (("host", H), ("gpu", G)):
                            pl = D[f][k].reshape(H16 // 2, Wc)
                            det[f"{k}_{name}_top"] = pl[cy0 - 1, cx0 - 1:cx0 + 8].tolist() if my else None
                            det[f"{k}_{name}_left"] = pl[cy0:cy0 + 8, cx0 - 1].tolist() if mx else None
                            det[f"{k}_{name}_blk"] = pl[cy0:cy0 + 8, cx0:cx0 + 8].tolist()
                    det["src_cr"] = cr[f, cy0:cy0 + 8, cx0:cx0 + 8].tolist()
                    det["src_cb"] = cb[f, cy0:cy0 + 8, cx0:cx0 + 8].tolist()
                    det["lv_host_c"] = H[f]["lv"][mb][256:].tolist()
                    det["lv_gpu_c"] = G[f]["lv"][mb][256:].tolist()
                    det["lv_host_y"] = H[f]["lv"][mb][:16].tolist()
                    det["lv_gpu_y"] = G[f]["lv"][mb][:16].tolist()
                    print(json.dumps(det), flush=True)
            print(json.dumps(rep), flush=True)
    _lib.lib().arb_set_h264_sync(1)


if __name__ == "__main__":
    main()
