"""Layer-by-layer G forward comparison, HIP vs CPU oracle (fp32 and fp64). Debug aid."""
import os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
import torch.nn.functional as F
from oracle import dsgan_cpu as O
from oracle.recipe import make_params, synth_pair
from models.mixconvnext import MixConvNeXtML
from dsgan_hip import functional as HF

recipe = sys.argv[1] if len(sys.argv) > 1 else "ref"
size = int(sys.argv[2]) if len(sys.argv) > 2 else 64
gp = make_params(O.g_param_spec(), recipe, 1000)
gp64 = make_params(O.g_param_spec(), recipe, 1000, torch.float64)
net = MixConvNeXtML().cuda()
with torch.no_grad():
    for k, v in net.state_dict().items():
        v.copy_(gp[k])
A, _ = synth_pair(1, size, 1)
x = A.cuda()

def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return ((a - b).norm() / max(b.norm().item(), 1e-30)).item()

def cmp(name, mine, f):
    r32 = f(gp, A)
    r64 = f(gp64, A.double())
    print("%-28s mine-vs-64 %.2e   ref32-vs-64 %.2e   |x|=%.3e" % (name, rel(mine, r64), rel(r32, r64), r64.abs().max().item()))

mp = lambda t: HF.max_pool2d(t, 2)
with torch.no_grad():
    R1 = net.c1(x)
    cmp("R1", R1, lambda p, a: O.block_fwd(p, "c1.", a))
    h = HF.dwconv(x, net.c1.dwconv.weight, net.c1.dwconv.bias)
    cmp("c1.dw", h, lambda p, a: F.conv2d(a, p["c1.dwconv.weight"], p["c1.dwconv.bias"], padding=3, groups=3))
    hn = HF.instance_norm(h)
    cmp("c1.dw.IN", hn, lambda p, a: F.instance_norm(F.conv2d(a, p["c1.dwconv.weight"], p["c1.dwconv.bias"], padding=3, groups=3)))
    loc = net.local(x)
    cmp("Loc", loc, lambda p, a: O.origin_mlka_fwd(p, a))
    d1 = HF.conv2d(x, net.local.to32.weight)
    m1 = net.local.mid32(mp(d1))
    cmp("local.mid32", m1, lambda p, a: O.midmlka_fwd(p, "local.mid32.", F.max_pool2d(F.conv2d(a, p["local.to32.weight"]), 2)))
    y = net(x)
    cmp("G out", y, lambda p, a: O.g_fwd(p, a))
