"""paddle.vision.ops against scalar loop oracles written from the reference kernels' definitions
(reference tests: test/legacy_test/test_yolo_box_op.py, test_yolov3_loss_op.py, test_prior_box_op.py,
test_box_coder_op.py, test_roi_align_op.py, test_roi_pool_op.py, test_psroi_pool_op.py, test_nms_op.py,
test_matrix_nms_op.py, test_generate_proposals_v2_op.py, test_distribute_fpn_proposals_op.py,
test_deformable_conv_op.py)."""
import math

import numpy as np
import pytest
import torch

import paddle2_amd as paddle
from paddle2_amd.vision import ops as V


def T(a, dt="float32"):
    return paddle.to_tensor(np.asarray(a, dtype=dt))


def sig(v):
    return 1.0 / (1.0 + math.exp(-v))


def test_yolo_box_matches_loop():
    rs = np.random.RandomState(0)
    an = [10, 13, 16, 30]
    cls = 3
    x = rs.randn(2, 2 * (5 + cls), 4, 4).astype("float32")
    img = np.array([[64, 80], [32, 48]], "int32")
    boxes, scores = V.yolo_box(T(x), T(img, "int32"), an, cls, 0.3, 8, clip_bbox=True, scale_x_y=1.2)
    boxes, scores = boxes.numpy(), scores.numpy()
    bias = -0.5 * 0.2
    for i in range(2):
        ih, iw = img[i]
        for j in range(2):
            for k in range(4):
                for l in range(4):
                    base = j * (5 + cls)
                    conf = sig(x[i, base + 4, k, l])
                    idx = j * 16 + k * 4 + l
                    if conf < 0.3:
                        assert np.all(boxes[i, idx] == 0) and np.all(scores[i, idx] == 0)
                        continue
                    cx = (l + sig(x[i, base, k, l]) * 1.2 + bias) * iw / 4
                    cy = (k + sig(x[i, base + 1, k, l]) * 1.2 + bias) * ih / 4
                    bw = math.exp(x[i, base + 2, k, l]) * an[2 * j] * iw / 32
                    bh = math.exp(x[i, base + 3, k, l]) * an[2 * j + 1] * ih / 32
                    ref = [max(cx - bw / 2, 0), max(cy - bh / 2, 0), min(cx + bw / 2, iw - 1), min(cy + bh / 2, ih - 1)]
                    np.testing.assert_allclose(boxes[i, idx], ref, rtol=1e-5, atol=1e-4)
                    for c in range(cls):
                        np.testing.assert_allclose(scores[i, idx, c], conf * sig(x[i, base + 5 + c, k, l]), rtol=1e-5)


def _sce(x, t):
    return max(x, 0) - x * t + math.log1p(math.exp(-abs(x)))


def _yolo_loss_loop(x, gtb, gtl, anchors, mask, cls, ignore, ds, smooth):
    n, _, h, w = x.shape
    an_num, m = len(anchors) // 2, len(mask)
    insz = ds * h
    pos, neg = (1 - min(1 / cls, 1 / 40), min(1 / cls, 1 / 40)) if smooth else (1.0, 0.0)
    loss = np.zeros(n)

    def iou(a, b):
        def ov(c1, w1, c2, w2):
            return min(c1 + w1 / 2, c2 + w2 / 2) - max(c1 - w1 / 2, c2 - w2 / 2)
        iw, ih = ov(a[0], a[2], b[0], b[2]), ov(a[1], a[3], b[1], b[3])
        inter = 0.0 if (iw < 0 or ih < 0) else iw * ih
        return inter / (a[2] * a[3] + b[2] * b[3] - inter)

    for i in range(n):
        obj = np.zeros((m, h, w))
        for j in range(m):
            for k in range(h):
                for l in range(w):
                    c = j * (5 + cls)
                    pb = [(l + sig(x[i, c, k, l])) / w, (k + sig(x[i, c + 1, k, l])) / h,
                          math.exp(x[i, c + 2, k, l]) * anchors[2 * mask[j]] / insz,
                          math.exp(x[i, c + 3, k, l]) * anchors[2 * mask[j] + 1] / insz]
                    best = 0.0
                    for t in range(gtb.shape[1]):
                        if gtb[i, t, 2] <= 0 or gtb[i, t, 3] <= 0:
                            continue
                        best = max(best, iou(pb, gtb[i, t]))
                    if best > ignore:
                        obj[j, k, l] = -1
        for t in range(gtb.shape[1]):
            g = gtb[i, t]
            if g[2] <= 0 or g[3] <= 0:
                continue
            gi, gj = int(g[0] * w), int(g[1] * h)
            ious = [iou([0, 0, anchors[2 * a] / insz, anchors[2 * a + 1] / insz], [0, 0, g[2], g[3]])
                    for a in range(an_num)]
            bn = int(np.argmax(ious))
            if bn not in mask:
                continue
            mi = mask.index(bn)
            c = mi * (5 + cls)
            sc = 2.0 - g[2] * g[3]
            loss[i] += _sce(x[i, c, gj, gi], g[0] * w - gi) * sc + _sce(x[i, c + 1, gj, gi], g[1] * h - gj) * sc
            loss[i] += abs(x[i, c + 2, gj, gi] - math.log(g[2] * insz / anchors[2 * bn])) * sc
            loss[i] += abs(x[i, c + 3, gj, gi] - math.log(g[3] * insz / anchors[2 * bn + 1])) * sc
            obj[mi, gj, gi] = 1.0
            for cc in range(cls):
                loss[i] += _sce(x[i, c + 5 + cc, gj, gi], pos if cc == gtl[i, t] else neg)
        for j in range(m):
            for k in range(h):
                for l in range(w):
                    o = obj[j, k, l]
                    v = x[i, j * (5 + cls) + 4, k, l]
                    if o > 1e-5:
                        loss[i] += _sce(v, 1.0) * o
                    elif o > -0.5:
                        loss[i] += _sce(v, 0.0)
    return loss


@pytest.mark.parametrize("smooth", [True, False])
def test_yolo_loss_matches_loop_and_backprops(smooth):
    rs = np.random.RandomState(1)
    anchors = [10, 13, 16, 30, 33, 23, 30, 61]
    mask = [1, 2]
    cls = 4
    x = (rs.randn(2, len(mask) * (5 + cls), 5, 5) * 0.5).astype("float32")
    gtb = np.array([[[0.3, 0.4, 0.2, 0.3], [0.7, 0.2, 0.35, 0.1], [0, 0, 0, 0]],
                    [[0.5, 0.5, 0.5, 0.6], [0.1, 0.9, 0.05, 0.08], [0.52, 0.48, 0.3, 0.5]]], "float32")
    gtl = np.array([[1, 3, 0], [2, 0, 1]], "int32")
    xt = T(x)
    xt.stop_gradient = False
    loss = V.yolo_loss(xt, T(gtb), T(gtl, "int32"), anchors, mask, cls, 0.6, 8, use_label_smooth=smooth)
    np.testing.assert_allclose(loss.numpy(), _yolo_loss_loop(x, gtb, gtl, anchors, mask, cls, 0.6, 8, smooth),
                               rtol=1e-4)
    loss.sum().backward()
    assert np.isfinite(xt.grad.numpy()).all() and np.abs(xt.grad.numpy()).sum() > 0


def test_prior_box_matches_loop():
    feat = paddle.zeros([1, 8, 3, 4])
    img = paddle.zeros([1, 3, 30, 40])
    boxes, var = V.prior_box(feat, img, [4.0, 8.0], [9.0, 12.0], [2.0, 0.5], flip=True, clip=True)
    b = boxes.numpy()
    ars = [1.0, 2.0, 0.5]   # 0.5 flip of 2.0 already present
    for hh in range(3):
        for ww in range(4):
            cx, cy = (ww + 0.5) * 10, (hh + 0.5) * 10
            exp = []
            for s, ms in enumerate([4.0, 8.0]):
                for ar in ars:
                    bw, bh = ms * math.sqrt(ar) / 2, ms / math.sqrt(ar) / 2
                    exp.append([(cx - bw) / 40, (cy - bh) / 30, (cx + bw) / 40, (cy + bh) / 30])
                v = math.sqrt(ms * [9.0, 12.0][s]) / 2
                exp.append([(cx - v) / 40, (cy - v) / 30, (cx + v) / 40, (cy + v) / 30])
            np.testing.assert_allclose(b[hh, ww], np.clip(exp, 0, 1), rtol=1e-5, atol=1e-6)
    assert list(var.shape) == list(boxes.shape) and np.allclose(var.numpy()[..., 2], 0.2)


def test_box_coder_encode_decode_roundtrip():
    rs = np.random.RandomState(2)
    pri = np.sort(rs.rand(5, 4).astype("float32") * 10, axis=1)[:, [0, 1, 2, 3]]
    pri[:, 2:] += 1
    tgt = pri[rs.randint(0, 5, 3)] + rs.rand(3, 4).astype("float32") * 0.3
    var = [0.1, 0.1, 0.2, 0.2]
    enc = V.box_coder(T(pri), var, T(tgt), "encode_center_size", box_normalized=False).numpy()
    # loop check of one entry
    i, j = 1, 3
    pw, ph = pri[j, 2] - pri[j, 0] + 1, pri[j, 3] - pri[j, 1] + 1
    tw, th = tgt[i, 2] - tgt[i, 0] + 1, tgt[i, 3] - tgt[i, 1] + 1
    ref = [((tgt[i, 0] + tgt[i, 2]) / 2 - (pri[j, 0] + pw / 2)) / pw / 0.1,
           ((tgt[i, 1] + tgt[i, 3]) / 2 - (pri[j, 1] + ph / 2)) / ph / 0.1,
           math.log(tw / pw) / 0.2, math.log(th / ph) / 0.2]
    np.testing.assert_allclose(enc[i, j], ref, rtol=1e-4)
    dec = V.box_coder(T(pri), var, T(enc), "decode_center_size", box_normalized=False).numpy()
    # the reference's pixel convention: encode takes the centre as (x1 + x2) / 2 while the width carries the
    # +1, so an un-normalized round trip lands half a pixel inside the original corners
    np.testing.assert_allclose(dec, np.broadcast_to(tgt[:, None] - 0.5, dec.shape), rtol=1e-4, atol=1e-4)
    enc_n = V.box_coder(T(pri), var, T(tgt), "encode_center_size", box_normalized=True)
    dec_n = V.box_coder(T(pri), var, enc_n, "decode_center_size", box_normalized=True).numpy()
    np.testing.assert_allclose(dec_n, np.broadcast_to(tgt[:, None], dec_n.shape), rtol=1e-4, atol=1e-4)
    dec2 = V.box_coder(T(pri), T(np.tile(np.array(var, "float32"), (5, 1))), T(enc), "decode_center_size",
                       box_normalized=False).numpy()
    np.testing.assert_allclose(dec2, dec, rtol=1e-6)


def _bilin(img, y, x):
    H, W = img.shape[-2:]
    if y < -1 or y > H or x < -1 or x > W:
        return np.zeros(img.shape[0])
    y, x = max(y, 0.0), max(x, 0.0)
    yl, xl = int(y), int(x)
    if yl >= H - 1:
        yh = yl = H - 1
        y = float(yl)
    else:
        yh = yl + 1
    if xl >= W - 1:
        xh = xl = W - 1
        x = float(xl)
    else:
        xh = xl + 1
    ly, lx = y - yl, x - xl
    return ((1 - ly) * (1 - lx) * img[:, yl, xl] + (1 - ly) * lx * img[:, yl, xh] + ly * (1 - lx) * img[:, yh, xl]
            + ly * lx * img[:, yh, xh])


@pytest.mark.parametrize("aligned,ratio", [(True, -1), (False, 2)])
def test_roi_align_matches_loop(aligned, ratio):
    rs = np.random.RandomState(3)
    x = rs.randn(2, 3, 9, 11).astype("float32")
    boxes = np.array([[1, 1, 6, 5], [0.5, 2.2, 10.3, 8.9], [3, 3, 3.5, 4]], "float32")
    bn = np.array([2, 1], "int32")
    out = V.roi_align(T(x), T(boxes), T(bn, "int32"), (2, 3), spatial_scale=0.8, sampling_ratio=ratio,
                      aligned=aligned).numpy()
    bid = [0, 0, 1]
    off = 0.5 if aligned else 0.0
    for r in range(3):
        x1, y1, x2, y2 = boxes[r] * 0.8 - off
        rw, rh = x2 - x1, y2 - y1
        if not aligned:
            rw, rh = max(rw, 1), max(rh, 1)
        gh = ratio if ratio > 0 else math.ceil(rh / 2)
        gw = ratio if ratio > 0 else math.ceil(rw / 3)
        for py in range(2):
            for px in range(3):
                acc = np.zeros(3)
                for iy in range(gh):
                    for ix in range(gw):
                        yy = y1 + rh / 2 * (py + (iy + 0.5) / gh)
                        xx = x1 + rw / 3 * (px + (ix + 0.5) / gw)
                        acc += _bilin(x[bid[r]], yy, xx)
                np.testing.assert_allclose(out[r, :, py, px], acc / (gh * gw), rtol=1e-4, atol=1e-5)


def test_roi_pool_and_psroi_pool_match_loops():
    rs = np.random.RandomState(4)
    x = rs.randn(1, 8, 7, 9).astype("float32")
    boxes = np.array([[1, 0, 7, 5], [2.4, 1.6, 3.1, 2.2]], "float32")
    out = V.roi_pool(T(x), T(boxes), T([2], "int32"), 2, spatial_scale=1.0).numpy()
    for r in range(2):
        sw, sh, ew, eh = [int(round(v)) for v in boxes[r]]
        bh, bw = max(eh - sh + 1, 1) / 2, max(ew - sw + 1, 1) / 2
        for ph in range(2):
            for pw in range(2):
                hs = min(max(int(math.floor(ph * bh)) + sh, 0), 7)
                he = min(max(int(math.ceil((ph + 1) * bh)) + sh, 0), 7)
                ws = min(max(int(math.floor(pw * bw)) + sw, 0), 9)
                we = min(max(int(math.ceil((pw + 1) * bw)) + sw, 0), 9)
                ref = x[0, :, hs:he, ws:we].max((1, 2)) if he > hs and we > ws else np.zeros(8)
                np.testing.assert_allclose(out[r, :, ph, pw], ref, rtol=1e-6)
    ps = V.psroi_pool(T(x), T(boxes), T([2], "int32"), 2, spatial_scale=0.5).numpy()
    assert ps.shape == (2, 2, 2, 2)
    for r in range(2):
        rb = np.round(boxes[r])
        x1, y1, x2, y2 = rb[0] * 0.5, rb[1] * 0.5, (rb[2] + 1) * 0.5, (rb[3] + 1) * 0.5
        rh, rw = max(y2 - y1, 0.1), max(x2 - x1, 0.1)
        for k in range(2):
            for ph in range(2):
                for pw in range(2):
                    hs = min(max(int(math.floor(ph * rh / 2 + y1)), 0), 7)
                    he = min(max(int(math.ceil((ph + 1) * rh / 2 + y1)), 0), 7)
                    ws = min(max(int(math.floor(pw * rw / 2 + x1)), 0), 9)
                    we = min(max(int(math.ceil((pw + 1) * rw / 2 + x1)), 0), 9)
                    ch = (k * 2 + ph) * 2 + pw
                    ref = x[0, ch, hs:he, ws:we].mean() if he > hs and we > ws else 0.0
                    np.testing.assert_allclose(ps[r, k, ph, pw], ref, rtol=1e-5, atol=1e-6)


def _np_nms(b, thr):
    keep, removed = [], np.zeros(len(b), bool)
    for i in range(len(b)):
        if removed[i]:
            continue
        keep.append(i)
        for j in range(i + 1, len(b)):
            iw = max(0, min(b[i, 2], b[j, 2]) - max(b[i, 0], b[j, 0]))
            ih = max(0, min(b[i, 3], b[j, 3]) - max(b[i, 1], b[j, 1]))
            inter = iw * ih
            u = (b[i, 2] - b[i, 0]) * (b[i, 3] - b[i, 1]) + (b[j, 2] - b[j, 0]) * (b[j, 3] - b[j, 1]) - inter
            if inter / u > thr:
                removed[j] = True
    return keep


def test_nms_variants():
    rs = np.random.RandomState(5)
    xy = rs.rand(40, 2) * 20
    wh = rs.rand(40, 2) * 8 + 1
    b = np.concatenate([xy, xy + wh], 1).astype("float32")
    s = rs.rand(40).astype("float32")
    assert V.nms(T(b), 0.4).numpy().tolist() == _np_nms(b, 0.4)
    order = np.argsort(-s, kind="stable")
    ref = order[_np_nms(b[order], 0.4)]
    assert V.nms(T(b), 0.4, T(s)).numpy().tolist() == ref.tolist()
    cat = rs.randint(0, 3, 40)
    got = V.nms(T(b), 0.4, T(s), T(cat, "int64"), [0, 1, 2], top_k=10).numpy()
    kept = []
    for c in range(3):
        idx = np.where(cat == c)[0]
        o = idx[np.argsort(-s[idx], kind="stable")]
        kept += o[_np_nms(b[o], 0.4)].tolist()
    kept = np.array(kept)
    ref = kept[np.argsort(-s[kept], kind="stable")][:10]
    assert got.tolist() == ref.tolist()


def test_matrix_nms_matches_loop():
    rs = np.random.RandomState(6)
    N, C, M = 2, 3, 12
    xy = rs.rand(N, M, 2)
    bb = np.concatenate([xy, xy + rs.rand(N, M, 2) * 0.4 + 0.05], -1).astype("float32")
    sc = rs.rand(N, C, M).astype("float32")
    out, rn, idx = V.matrix_nms(T(bb), T(sc), 0.2, 0.3, nms_top_k=8, keep_top_k=10, use_gaussian=False,
                                background_label=0, return_index=True)
    out, rn, idx = out.numpy(), rn.numpy(), idx.numpy()

    def iou(a, b):
        if b[0] > a[2] or b[2] < a[0] or b[1] > a[3] or b[3] < a[1]:
            return 0.0
        iw, ih = min(a[2], b[2]) - max(a[0], b[0]), min(a[3], b[3]) - max(a[1], b[1])
        inter = iw * ih
        return inter / ((a[2] - a[0]) * (a[3] - a[1]) + (b[2] - b[0]) * (b[3] - b[1]) - inter)

    ref_rows, ref_num = [], []
    for i in range(N):
        dets = []
        for c in range(1, C):
            cand = [k for k in range(M) if sc[i, c, k] > 0.2]
            cand = sorted(cand, key=lambda k: -sc[i, c, k])[:8]
            if not cand:
                continue
            ioum = np.zeros((len(cand), len(cand)))
            for a in range(len(cand)):
                for bq in range(a):
                    ioum[a, bq] = iou(bb[i, cand[a]], bb[i, cand[bq]])
            imax = [ioum[a, :a].max() if a else 0.0 for a in range(len(cand))]
            for a in range(len(cand)):
                d = min([1.0] + [(1 - ioum[a, bq]) / (1 - imax[bq]) for bq in range(a)])
                ds = d * sc[i, c, cand[a]]
                if ds > 0.3:
                    dets.append((ds, c, cand[a]))
        dets = sorted(dets, key=lambda t: -t[0])[:10]
        ref_num.append(len(dets))
        ref_rows += [[c, ds, *bb[i, k]] for ds, c, k in dets]
    assert rn.tolist() == ref_num
    np.testing.assert_allclose(out, np.array(ref_rows, "float32").reshape(-1, 6), rtol=1e-5, atol=1e-6)
    assert idx.shape == (sum(ref_num), 1)


def test_generate_proposals_and_distribute_fpn():
    rs = np.random.RandomState(7)
    N, A, H, W = 2, 3, 4, 5
    scores = rs.rand(N, A, H, W).astype("float32")
    deltas = (rs.randn(N, 4 * A, H, W) * 0.2).astype("float32")
    anchors = np.zeros((H, W, A, 4), "float32")
    for h in range(H):
        for w in range(W):
            for a in range(A):
                s = 8 * (a + 1)
                anchors[h, w, a] = [w * 8, h * 8, w * 8 + s, h * 8 + s]
    var = np.ones((H, W, A, 4), "float32")
    img = np.array([[40, 48], [36, 44]], "float32")
    rois, probs, num = V.generate_proposals(T(scores), T(deltas), T(img), T(anchors), T(var), pre_nms_top_n=30,
                                            post_nms_top_n=10, nms_thresh=0.6, min_size=2.0, return_rois_num=True)
    rois, probs, num = rois.numpy(), probs.numpy(), num.numpy()
    assert rois.shape[0] == num.sum() and (num <= 10).all() and (num >= 1).all()
    start = 0
    for i in range(N):
        r = rois[start:start + num[i]]
        p = probs[start:start + num[i], 0]
        assert np.all(np.diff(p) <= 1e-7)                       # descending scores
        assert (r[:, 0] >= 0).all() and (r[:, 2] <= img[i, 1]).all() and (r[:, 3] <= img[i, 0]).all()
        # survivors pairwise below the NMS threshold
        for a in range(len(r)):
            for b in range(a):
                iw = max(0, min(r[a, 2], r[b, 2]) - max(r[a, 0], r[b, 0]))
                ih = max(0, min(r[a, 3], r[b, 3]) - max(r[a, 1], r[b, 1]))
                inter = iw * ih
                u = (r[a, 2] - r[a, 0]) * (r[a, 3] - r[a, 1]) + (r[b, 2] - r[b, 0]) * (r[b, 3] - r[b, 1]) - inter
                assert inter / u <= 0.6 + 1e-6
        start += num[i]
    multi, restore, per_level = V.distribute_fpn_proposals(T(rois), 2, 5, 4, 224, rois_num=T(num, "int32"))
    cat = np.concatenate([m.numpy() for m in multi])
    np.testing.assert_allclose(cat[restore.numpy()[:, 0]], rois)
    assert sum(int(p.numpy().sum()) for p in per_level) == rois.shape[0]
    for L, m in zip(range(2, 6), multi):
        mm = m.numpy()
        if len(mm):
            sc_ = np.sqrt((mm[:, 2] - mm[:, 0]) * (mm[:, 3] - mm[:, 1]))
            lv = np.clip(np.floor(np.log2(sc_ / 224 + 1e-6) + 4), 2, 5)
            assert (lv == L).all()


def test_deform_conv2d():
    rs = np.random.RandomState(8)
    x = rs.randn(2, 4, 6, 7).astype("float32")
    w = rs.randn(6, 2, 3, 3).astype("float32")
    b = rs.randn(6).astype("float32")
    zero_off = np.zeros((2, 2 * 9, 6, 7), "float32")
    out = V.deform_conv2d(T(x), T(zero_off), T(w), T(b), padding=1, groups=2).numpy()
    ref = torch.nn.functional.conv2d(torch.tensor(x), torch.tensor(w), torch.tensor(b), padding=1, groups=2).numpy()
    np.testing.assert_allclose(out, ref, rtol=1e-4, atol=1e-4)
    # a constant integer offset of (+1, -1) equals convolving the shifted image
    off = np.zeros((2, 9, 2, 6, 7), "float32")
    off[:, :, 0] = 1.0
    off[:, :, 1] = -1.0
    out2 = V.deform_conv2d(T(x), T(off.reshape(2, 18, 6, 7)), T(w), None, padding=1, groups=2).numpy()
    # oracle: tap (ky, kx) of output (oy, ox) reads x[oy - 1 + ky + 1, ox - 1 + kx - 1] (zero outside)
    xp = np.pad(x, ((0, 0), (0, 0), (2, 2), (2, 2)))
    ref2 = np.zeros((2, 6, 6, 7), "float32")
    for ky in range(3):
        for kx in range(3):
            patch = xp[:, :, 2 + ky:2 + ky + 6, kx:kx + 7]          # rows oy + ky, cols ox + kx - 2
            for g in range(2):
                ref2[:, 3 * g:3 * g + 3] += np.einsum("oc,nchw->nohw", w[3 * g:3 * g + 3, :, ky, kx],
                                                      patch[:, 2 * g:2 * g + 2])
    np.testing.assert_allclose(out2, ref2, rtol=1e-4, atol=1e-4)
    # v2 mask of 0.5 halves the output; gradients flow to input, offset and mask
    mask = np.full((2, 9, 6, 7), 0.5, "float32")
    xt, ot, mt = T(x), T(rs.randn(2, 18, 6, 7).astype("float32") * 0.3), T(mask)
    for t in (xt, ot, mt):
        t.stop_gradient = False
    y = V.deform_conv2d(xt, ot, T(w), None, padding=1, groups=2, mask=mt)
    y.sum().backward()
    assert all(np.isfinite(t.grad.numpy()).all() for t in (xt, ot, mt))
    layer = V.DeformConv2D(4, 6, 3, padding=1, groups=2)
    assert list(layer(T(x), T(zero_off)).shape) == [2, 6, 6, 7]


def test_read_file_decode_jpeg(tmp_path):
    from PIL import Image

    yy, xx = np.mgrid[0:12, 0:16]
    arr = np.stack([yy * 20, xx * 15, (yy + xx) * 8], -1).astype("uint8")     # smooth: JPEG-friendly
    p = tmp_path / "a.jpg"
    Image.fromarray(arr).save(p, quality=95)
    data = V.read_file(str(p))
    assert data.numpy().dtype == np.uint8 and data.numpy().size == p.stat().st_size
    img = V.decode_jpeg(data, mode="rgb").numpy()
    assert img.shape == (3, 12, 16) and np.abs(img.astype(int) - arr.transpose(2, 0, 1)).mean() < 12
    assert V.decode_jpeg(data, mode="gray").numpy().shape == (1, 12, 16)


def test_layers_and_conv_norm_act():
    x = T(np.random.RandomState(10).randn(1, 8, 10, 10))
    boxes, bn = T([[1, 1, 8, 8]]), T([1], "int32")
    assert list(V.RoIAlign(3)(x, boxes, bn).shape) == [1, 8, 3, 3]
    assert list(V.RoIPool(2)(x, boxes, bn).shape) == [1, 8, 2, 2]
    assert list(V.PSRoIPool(2)(x, boxes, bn).shape) == [1, 2, 2, 2]
    cna = V.ConvNormActivation(8, 4, 3)
    assert list(cna(x).shape) == [1, 4, 10, 10]
