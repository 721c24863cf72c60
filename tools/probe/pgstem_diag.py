"""PatchGAN D forward + backward with the stem kernels on / off (fp32 mode), per-parameter gradient
differences, plus a float64 torch reference of the same D (probe for the 256^2 step test)."""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import functools  # noqa: E402

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

import dsgan_hip  # noqa: E402
from dsgan_hip import functional as HF  # noqa: E402
from models.networks import NLayerDiscriminator  # noqa: E402


def ref_d(D, x):
    h = x
    for idx, stride, use_in in D.plan:
        c = D.model[idx]
        h = F.conv2d(h, c.weight.double(), None if c.bias is None else c.bias.double(), stride=stride, padding=1)
        if use_in is None:
            return h
        if use_in:
            h = F.instance_norm(h, eps=1e-5)
        h = F.leaky_relu(h, 0.2)
    return h


def main():
    dsgan_hip.require_gpu()
    HF.set_precision(os.environ.get("PREC", "fp32"))
    torch.manual_seed(0)
    norm = functools.partial(torch.nn.InstanceNorm2d, affine=False, track_running_stats=False)
    D = NLayerDiscriminator(6, 32, 3, norm_layer=norm).cuda()
    for p in D.parameters():
        torch.nn.init.normal_(p, 0.0, 0.05)
    g = torch.Generator().manual_seed(1)
    x = torch.randn(2, 6, 256, 256, generator=g).cuda()
    r = None
    res = {}
    for on in (True, False):
        HF.PGSTEM[0] = on
        for p in D.parameters():
            p.grad = torch.zeros_like(p)
        h = x
        acts = []
        for idx, stride, use_in in D.plan:
            c = D.model[idx]
            if use_in is None:
                h = HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1)
            elif use_in:
                h = HF.instance_norm(HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1), act="lrelu")
            else:
                h = HF.conv2d(h, c.weight, c.bias, stride=stride, pad=1, act="lrelu")
            h.retain_grad()
            acts.append(h)
        out = h
        if r is None:
            r = torch.randn(out.shape, generator=g).cuda()
        (out * r).sum().backward()
        torch.cuda.synchronize()
        res[on] = (out.detach().clone(), {k: p.grad.detach().clone() for k, p in D.named_parameters()},
                   [a.detach().clone() for a in acts], [a.grad.detach().clone() for a in acts])
    for i in range(len(res[True][2])):
        a0, a1 = res[True][2][i], res[False][2][i]
        g0, g1 = res[True][3][i], res[False][3][i]
        print("layer %d act on/off %.3e  grad on/off %.3e" % (i, ((a0 - a1).norm() / a1.norm()).item(),
                                                             ((g0 - g1).norm() / g1.norm()).item()))
    xd = x.double().cpu()
    # float64 reference with the same parameters
    Dc = NLayerDiscriminator(6, 32, 3, norm_layer=norm)
    Dc.load_state_dict({k: v.cpu() for k, v in D.state_dict().items()})
    Dc = Dc.double()
    for p in Dc.parameters():
        p.grad = None
    od = ref_d(Dc, xd)
    (od * r.double().cpu()).sum().backward()
    print("out on/off rel %.3e  on/ref %.3e  off/ref %.3e" % (
        ((res[True][0] - res[False][0]).norm() / res[False][0].norm()).item(),
        ((res[True][0].double().cpu() - od.detach()).norm() / od.norm()).item(),
        ((res[False][0].double().cpu() - od.detach()).norm() / od.norm()).item()))
    for k, p in Dc.named_parameters():
        a, b = res[True][1][k].double().cpu(), res[False][1][k].double().cpu()
        q = p.grad
        print("%-18s on/off %.3e  on/ref %.3e  off/ref %.3e  |g| %.3e" % (
            k, ((a - b).norm() / b.norm()).item(), ((a - q).norm() / q.norm()).item(),
            ((b - q).norm() / q.norm()).item(), q.norm().item()))


if __name__ == "__main__":
    main()
