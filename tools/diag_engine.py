"""Per-stage comparison of the HIP engine against a decomposed fp32 reference (forward tensors + activation grads).

Run on a GPU box:  python tools/diag_engine.py [S] [B]
"""
import os
import sys

import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from crack_detection_federatedlearning_grpc_amd.data.device import make_synthetic_device  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models import unet_ref as R  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.engine import UNetEngine  # noqa: E402
from crack_detection_federatedlearning_grpc_amd.models.spec import DEC_FILTERS, ENC_FILTERS, ParamTable  # noqa: E402


def bfv(t):
    return t.view(torch.bfloat16).float().cpu()


def rel(a, b):
    return float((a - b).norm() / (b.norm() + 1e-12))


def main(S=64, B=2):
    table = ParamTable()
    data = make_synthetic_device(max(8, B), S, seed=0)   # idx 0..B-1 must be bound images
    eng = UNetEngine(table, B, S)
    eng.bind_data(data.images, data.masks)
    flat = table.init_flat(0)
    eng.set_flat(flat)
    eng.idx.copy_(torch.arange(B, dtype=torch.int32, device=eng.dev))
    eng._zero_step()
    eng.forward(True)
    eng.backward()
    torch.cuda.synchronize()
    A, D = eng.act, eng.dg
    x = data.images[:B].float().cpu() / 255.0
    y = data.masks[:B].float().cpu()[..., None]
    p = torch.as_tensor(flat)
    P = lambda l, w: R._p(p, table, l, w)  # noqa: E731
    names = eng.names
    keep = {}

    def nhwc(t):
        return t.permute(0, 2, 3, 1)

    def bn(t, name):
        return R.batchnorm_train(t, P(name, "gamma"), P(name, "beta"), P(name, "moving_mean"),
                                 P(name, "moving_variance"), 0.99, 1e-3)[0]

    xin = nhwc(x).permute(0, 3, 1, 2) if False else x.permute(0, 3, 1, 2)
    y0 = R.conv2d_same(xin, P(names[0], "kernel"), P(names[0], "bias"), 2)
    keep["y0"] = y0
    a0 = F.relu(bn(y0, names[1]))
    xcur = a0
    for k in range(3):
        s1, b1, s2, b2, rc = names[2 + 5 * k:7 + 5 * k]
        t = F.relu(xcur)
        c = t.shape[1]
        d1 = F.conv2d(F.pad(t, (1, 1, 1, 1)), P(s1, "depthwise_kernel").permute(2, 3, 0, 1), None, groups=c)
        keep[f"e{k}_d1"] = d1
        y1 = F.conv2d(d1, P(s1, "pointwise_kernel").permute(3, 2, 0, 1), P(s1, "bias"))
        keep[f"e{k}_y1"] = y1
        t = F.relu(bn(y1, b1))
        d2 = F.conv2d(F.pad(t, (1, 1, 1, 1)), P(s2, "depthwise_kernel").permute(2, 3, 0, 1), None, groups=t.shape[1])
        keep[f"e{k}_d2"] = d2
        y2 = F.conv2d(d2, P(s2, "pointwise_kernel").permute(3, 2, 0, 1), P(s2, "bias"))
        keep[f"e{k}_y2"] = y2
        res = R.conv2d_same(xcur, P(rc, "kernel"), P(rc, "bias"), 2)
        keep[f"e{k}_res"] = res
        xn = R.maxpool_same(bn(y2, b2)) + res
        xn.retain_grad() if xn.requires_grad else None
        keep[f"e{k}_x"] = xn
        xcur = xn
    prev = xcur
    for k in range(4):
        t1, b1, t2, b2, rc = names[17 + 5 * k:22 + 5 * k]
        xin_ = prev if k == 0 else R.upsample2(prev)
        c1 = R.convt_same(F.relu(xin_), P(t1, "kernel"), P(t1, "bias"))
        keep[f"d{k}_c1"] = c1
        c2 = R.convt_same(F.relu(bn(c1, b1)), P(t2, "kernel"), P(t2, "bias"))
        keep[f"d{k}_c2"] = c2
        q = R.conv2d_same(prev, P(rc, "kernel"), P(rc, "bias"), 1)
        keep[f"d{k}_q"] = q
        xlo = bn(c2, b2) + (q if k == 0 else R.upsample2(q))
        keep[f"d{k}_xlo"] = xlo
        prev = xlo
    # forward compare
    for kname, t in keep.items():
        print(f"fwd {kname:10s} rel {rel(bfv(A[kname]), nhwc(t).detach()):.4f}")
    # gradients: rebuild with grad tracking of the stored intermediate tensors
    leaves = {}
    pq = p.clone().requires_grad_(True)
    logits, _ = R.unet_forward(pq, x, table)
    loss = R.bce_with_logits_mean(logits, y)
    # activation-grad comparisons via autograd.grad on recomputed graph
    Pq = lambda l, w: R._p(pq, table, l, w)  # noqa: E731

    def bnq(t, name):
        return R.batchnorm_train(t, Pq(name, "gamma"), Pq(name, "beta"), Pq(name, "moving_mean"),
                                 Pq(name, "moving_variance"), 0.99, 1e-3)[0]
    y0 = R.conv2d_same(x.permute(0, 3, 1, 2), Pq(names[0], "kernel"), Pq(names[0], "bias"), 2)
    xcur = F.relu(bnq(y0, names[1]))
    xs = []
    for k in range(3):
        s1, b1, s2, b2, rc = names[2 + 5 * k:7 + 5 * k]
        t = R.sepconv_same(F.relu(xcur), Pq(s1, "depthwise_kernel"), Pq(s1, "pointwise_kernel"), Pq(s1, "bias"))
        t = R.sepconv_same(F.relu(bnq(t, b1)), Pq(s2, "depthwise_kernel"), Pq(s2, "pointwise_kernel"), Pq(s2, "bias"))
        xcur = R.maxpool_same(bnq(t, b2)) + R.conv2d_same(xcur, Pq(rc, "kernel"), Pq(rc, "bias"), 2)
        xs.append(xcur)
    prev = xcur
    xlos = []
    for k in range(4):
        t1, b1, t2, b2, rc = names[17 + 5 * k:22 + 5 * k]
        xin_ = prev if k == 0 else R.upsample2(prev)
        c1 = R.convt_same(F.relu(xin_), Pq(t1, "kernel"), Pq(t1, "bias"))
        c2 = R.convt_same(F.relu(bnq(c1, b1)), Pq(t2, "kernel"), Pq(t2, "bias"))
        q = R.conv2d_same(prev, Pq(rc, "kernel"), Pq(rc, "bias"), 1)
        prev = bnq(c2, b2) + (q if k == 0 else R.upsample2(q))
        xlos.append(prev)
    hl = names[-1]
    lg = R.conv2d_same(R.upsample2(prev), Pq(hl, "kernel"), Pq(hl, "bias"), 1).permute(0, 2, 3, 1)
    loss2 = R.bce_with_logits_mean(lg, y)
    if os.environ.get("EMU"):
        # same graph with bf16 rounding (straight-through) at every point where the engine stores / feeds MFMA
        def r(t):
            return t + (t.to(torch.bfloat16).float() - t).detach()
        y0 = r(R.conv2d_same(x.permute(0, 3, 1, 2), Pq(names[0], "kernel"), Pq(names[0], "bias"), 2))
        xcur = F.relu(bnq(y0, names[1]))
        xs, xlos = [], []
        for k in range(3):
            s1, b1, s2, b2, rc = names[2 + 5 * k:7 + 5 * k]
            c = xcur.shape[1]
            d1 = r(F.conv2d(F.pad(F.relu(xcur), (1, 1, 1, 1)), Pq(s1, "depthwise_kernel").permute(2, 3, 0, 1), None,
                            groups=c))
            y1 = r(F.conv2d(d1, r(Pq(s1, "pointwise_kernel")).permute(3, 2, 0, 1), Pq(s1, "bias")))
            t = F.relu(bnq(y1, b1))
            d2 = r(F.conv2d(F.pad(t, (1, 1, 1, 1)), Pq(s2, "depthwise_kernel").permute(2, 3, 0, 1), None,
                            groups=t.shape[1]))
            y2 = r(F.conv2d(d2, r(Pq(s2, "pointwise_kernel")).permute(3, 2, 0, 1), Pq(s2, "bias")))
            res = r(R.conv2d_same(r(xcur), r(Pq(rc, "kernel")), Pq(rc, "bias"), 2))
            xcur = r(R.maxpool_same(bnq(y2, b2)) + res)
            xs.append(xcur)
        prev = xcur
        for k in range(4):
            t1, b1, t2, b2, rc = names[17 + 5 * k:22 + 5 * k]
            xin_ = prev if k == 0 else R.upsample2(prev)
            c1 = r(R.convt_same(F.relu(xin_), r(Pq(t1, "kernel")), Pq(t1, "bias")))
            c2 = r(R.convt_same(r(F.relu(bnq(c1, b1))), r(Pq(t2, "kernel")), Pq(t2, "bias")))
            q = r(R.conv2d_same(prev, r(Pq(rc, "kernel")), Pq(rc, "bias"), 1))
            prev = r(bnq(c2, b2) + (q if k == 0 else R.upsample2(q)))
            xlos.append(prev)
        print(f"emulated-bf16 fwd: xlo3 rel {rel(bfv(A['d3_xlo']), nhwc(prev).detach()):.4f} "
              f"x3 rel {rel(bfv(A['e2_x']), nhwc(xs[2]).detach()):.4f}")
        lg = R.conv2d_same(R.upsample2(prev), Pq(hl, "kernel"), Pq(hl, "bias"), 1).permute(0, 2, 3, 1)
        loss2 = R.bce_with_logits_mean(lg, y)
    print(f"loss ref {float(loss):.5f} decomposed {float(loss2):.5f} engine {eng.read_metrics('train')['loss']:.5f}")
    grads = torch.autograd.grad(loss2, xs + xlos + [pq])
    gx, gxlo, gp = grads[:3], grads[3:7], grads[7]
    print(f"grad xlo3 rel {rel(bfv(D['dxlo3']), nhwc(gxlo[3])):.4f}")
    for k in range(3, 0, -1):
        print(f"grad xlo{k - 1} rel {rel(bfv(D[f'd{k}_dprev']), nhwc(gxlo[k - 1])):.4f}")
    print(f"grad x3 (e2_x) rel {rel(bfv(D['d0_dprev']), nhwc(gx[2])):.4f}")
    for k in range(2, 0, -1):
        print(f"grad e{k - 1}_x rel {rel(bfv(D[f'e{k}_dx']), nhwc(gx[k - 1])):.4f}")
    ge = eng.grad.cpu()
    for e in table.entries:
        if not e.trainable:
            continue
        a, b = ge[e.offset:e.offset + e.size], gp[e.offset:e.offset + e.size]
        cos = float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-20))
        print(f"param {e.keras_name:45s} cos {cos:.4f} rel {rel(a, b):.4f} |ref| {float(b.norm()):.3e}")


if __name__ == "__main__":
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    main(S, B)
