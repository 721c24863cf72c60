"""MixConvNeXtML generator on libdsgan_hip.so (DSGAN/models/model/MixConvNeXtML.py).

Module tree, attribute names, parameter shapes and registration order are those of the
reference, so ``state_dict()`` keys match key-for-key (188 tensors) and reference checkpoints
load as-is.  The torch ``nn.Conv2d`` / ``nn.Linear`` / ``nn.ConvTranspose2d`` / ``nn.PReLU``
children are parameter *holders* only (their torch forward is never called): every forward
below is a chain of fused HIP kernels from ``dsgan_hip.functional``.
"""
import torch
import torch.nn as nn

from dsgan_hip import functional as HF


class CA(nn.Module):
    """Channel attention, MixConvNeXtML.py:5-22 (computed inside HF.mid_tail)."""

    def __init__(self, in_planes, ratio=8):
        super().__init__()
        self.fc1 = nn.Conv2d(in_planes, in_planes // ratio, 1, bias=False)
        self.relu1 = nn.PReLU()
        self.fc2 = nn.Conv2d(in_planes // ratio, in_planes, 1, bias=False)


class upSample(nn.Module):
    """ConvT 3x3/s2 -> IN -> GELU, then cat(skip) (MixConvNeXtML.py:48-66)."""

    def __init__(self, in_channel, out_channel):
        super().__init__()
        self.model = nn.Sequential(nn.ConvTranspose2d(in_channel, out_channel, kernel_size=3, stride=2,
                                                      padding=1, output_padding=1))

    def forward(self, x, feature_map, slot=None):
        t = self.model[0]
        return HF.convt_norm(x, t.weight, t.bias, feature_map, act="gelu", cat=True, slot=slot)


class MidMLKA(nn.Module):
    """MixConvNeXtML.py:76-117: chunk4 -> dw3/5/7/9 -> 1x1(+b) -> *CA -> IN -> +x -> GELU."""

    conv_precision = "fp32"

    def __init__(self, dim):
        super().__init__()
        self.dim = dim
        self.conv = nn.Conv2d(dim, dim, kernel_size=1)
        self.attn = CA(dim)
        q = dim // 4
        self.X3 = nn.Conv2d(q, q, 3, 1, 1, groups=q)
        self.X5 = nn.Conv2d(q, q, 5, 1, 2, groups=q)
        self.X7 = nn.Conv2d(q, q, 7, 1, 3, groups=q)
        self.X9 = nn.Conv2d(q, q, 9, 1, 4, groups=q)

    def forward(self, x):
        x = HF.share(x)   # read by the depthwise convs and by the residual of the tail
        d = HF.multi_dwconv(x, self.X3.weight, self.X3.bias, self.X5.weight, self.X5.bias,
                            self.X7.weight, self.X7.bias, self.X9.weight, self.X9.bias)
        # The 1x1 conv feeds an InstanceNorm whose input variance is far below eps at the
        # reference init: bf16 operand rounding there is amplified into the
        # branch output (tools/quality_diag.py: rel-l2 of fake_B after 10 steps 1.1 in bf16 vs
        # 0.05 with this conv in fp32), so it always runs with exact fp32 MFMA operands.
        with HF.precision(self.conv_precision):
            v = HF.conv2d(d, self.conv.weight, self.conv.bias)
        return HF.mid_tail(v, x, self.attn.fc1.weight, self.attn.relu1.weight, self.attn.fc2.weight)


class OriginMLKA(nn.Module):
    """The local (MLKA U-Net) branch, MixConvNeXtML.py:119-189."""

    def __init__(self):
        super().__init__()
        self.to32 = nn.Conv2d(3, 32, kernel_size=1, bias=False)
        self.mid32 = MidMLKA(32)
        self.to64 = nn.Conv2d(32, 64, kernel_size=1, bias=False)
        self.mid64 = MidMLKA(64)
        self.to128 = nn.Conv2d(64, 128, kernel_size=1, bias=False)
        self.mid128 = MidMLKA(128)
        self.to256 = nn.Conv2d(128, 256, kernel_size=1, bias=False)
        self.mid256 = MidMLKA(256)
        self.up1 = upSample(256, 128)
        self.upc1 = nn.Sequential(nn.Conv2d(256, 128, kernel_size=1, bias=False), MidMLKA(128))
        self.up2 = upSample(128, 64)
        self.upc2 = MidMLKA(128)
        self.up3 = upSample(128, 64)
        self.upc3 = MidMLKA(128)
        self.up4 = nn.Sequential(nn.ConvTranspose2d(128, 64, kernel_size=3, stride=2, padding=1,
                                                    output_padding=1))
        self.shortcut = nn.Sequential(nn.Conv2d(3, 64, 1, bias=False))

    def forward(self, x):
        mp = lambda t: HF.max_pool2d(t, 2)
        d1 = HF.conv2d(x, self.to32.weight)
        d2 = self.mid32(mp(d1))
        d3 = HF.share(HF.conv2d(d2, self.to64.weight))     # also the skip of up3
        d4 = HF.share(self.mid64(mp(d3)))                   # also the skip of up2
        d5 = HF.conv2d(d4, self.to128.weight)
        d6 = HF.share(self.mid128(mp(d5)))                  # also the skip of up1
        d7 = HF.conv2d(d6, self.to256.weight)
        d8 = self.mid256(mp(d7))
        u1 = self.upc1[1](HF.conv2d(self.up1(d8, d6), self.upc1[0].weight))
        u2 = self.upc2(self.up2(u1, d4))
        u3 = self.upc3(self.up3(u2, d3))
        sc = HF.instance_norm(HF.conv2d(x, self.shortcut[0].weight))
        t = self.up4[0]
        # GELU(IN(up4(u3)) + IN(shortcut(x))): the add and GELU are fused into the second IN
        return HF.convt_norm(u3, t.weight, t.bias, sc, act="gelu")


class Block(nn.Module):
    """ConvNeXt block, MixConvNeXtML.py:203-243:
    dw7x7(+b) -> IN -> Linear(C,4C)+b -> GELU -> Linear(4C,P)+b, + 1x1 shortcut(x)."""

    def __init__(self, dim, plans):
        super().__init__()
        self.shortcut = nn.Conv2d(dim, plans, kernel_size=1, bias=False)
        self.dwconv = nn.Conv2d(dim, dim, kernel_size=7, padding=3, groups=dim)
        self.pwconv1 = nn.Linear(dim, 4 * dim)
        self.pwconv2 = nn.Linear(4 * dim, plans)

    def forward(self, x, slot=None, acc=None):
        x = HF.share(x)   # read by the depthwise conv and by the 1x1 shortcut
        # norm=True: the block's InstanceNorm runs inside the MLP node (bf16 h, see PwMlpFn)
        d = HF.dwconv(x, self.dwconv.weight, self.dwconv.bias)
        return HF.pw_mlp(d, x, self.pwconv1.weight, self.pwconv1.bias, self.pwconv2.weight,
                         self.pwconv2.bias, self.shortcut.weight, norm=True, slot=slot, acc=acc)


def _skip(cin, cout, k):
    # nn.Sequential(MaxPool2d(k), Conv2d 1x1, InstanceNorm2d, GELU): only index 1 holds params
    return nn.Sequential(nn.MaxPool2d(kernel_size=k), nn.Conv2d(cin, cout, 1, bias=False),
                         nn.InstanceNorm2d(cout), nn.GELU())


def _skip_fwd(seq, x, pooled=None):
    """MaxPool(k) -> 1x1 -> IN -> GELU; ``pooled`` = MaxPool(k)(x) when already computed."""
    k = seq[0].kernel_size
    p = pooled if pooled is not None else HF.max_pool2d(x, k)
    return HF.instance_norm(HF.conv2d(p, seq[1].weight), act="gelu")


class downSkip(nn.Module):
    def __init__(self):
        super().__init__()
        self.to2, self.to4, self.to8, self.to16 = _skip(64, 128, 2), _skip(64, 256, 4), _skip(64, 512, 8), _skip(64, 1024, 16)

    def forward(self, x, pools=(None,) * 4):
        return [_skip_fwd(s, x, p) for s, p in zip((self.to2, self.to4, self.to8, self.to16), pools)]


class downSkip128(nn.Module):
    def __init__(self):
        super().__init__()
        self.to4, self.to8, self.to16 = _skip(128, 256, 2), _skip(128, 512, 4), _skip(128, 1024, 8)

    def forward(self, x, pools=(None,) * 3):
        return [_skip_fwd(s, x, p) for s, p in zip((self.to4, self.to8, self.to16), pools)]


class downSkip256(nn.Module):
    def __init__(self):
        super().__init__()
        self.to8, self.to16 = _skip(256, 512, 2), _skip(256, 1024, 4)

    def forward(self, x, pools=(None,) * 2):
        return [_skip_fwd(s, x, p) for s, p in zip((self.to8, self.to16), pools)]


class downSkip512(nn.Module):
    def __init__(self):
        super().__init__()
        self.to16 = _skip(512, 1024, 2)

    def forward(self, x, pools=(None,)):
        return [_skip_fwd(self.to16, x, pools[0])]


class MixConvNeXtML(nn.Module):
    """MixConvNeXtML.py:428-494 -- default generator (--which_model_netG MixConvNeXtML)."""

    def __init__(self):
        super().__init__()
        self.c1 = Block(3, 64)
        self.c2 = Block(64, 128)
        self.c3 = Block(128, 256)
        self.c4 = Block(256, 512)
        self.c5 = Block(512, 1024)
        self.u1 = upSample(1024, 512)
        self.uc1 = Block(1024, 512)
        self.u2 = upSample(512, 256)
        self.uc2 = Block(512, 256)
        self.u3 = upSample(256, 128)
        self.uc3 = Block(256, 128)
        self.u4 = upSample(128, 64)
        self.uc4 = Block(128, 64)
        self.down64 = downSkip()
        self.down128 = downSkip128()
        self.down256 = downSkip256()
        self.down512 = downSkip512()
        self.local = OriginMLKA()
        self.res = nn.Conv2d(64, 3, kernel_size=3, padding=1)

    def backward_order(self):
        """Children in the order backward_G finishes their weight-grads (the reverse of the
        forward's creation order: the local branch and the head are created last); FlatParams
        lays the G gradient buffer out in this order for the overlapped bucketed all-reduce."""
        return [self.res, self.local, self.uc4, self.u4, self.uc3, self.u3, self.uc2, self.u2, self.uc1, self.u1,
                self.down512, self.down256, self.down128, self.down64, self.c5, self.c4, self.c3, self.c2, self.c1]

    def forward(self, x):
        # R1..R4 feed the next stage's MaxPool(2), their skip pyramid and a decoder concat.  Every
        # MaxPool of R_i -- the encoder's k=2 (also the pyramid's k=2 branch) and the skips' k=4/8/16 --
        # comes from ONE pass over R_i (HF.max_pool_pyramid), whose backward adds all their grads
        # into R_i's in one pass.  Shared tensors accumulate their grads in one buffer (HF.share)
        # instead of through autograd adds.
        # The decoder concatenations cat(upSample head, R_i) are allocated up front: c_i writes R_i
        # straight into its tail and u_i only fills the head (no copy of the skip, HF.CatSlot).
        sh = HF.share

        def pyr(t, levels):   # [share(MaxPool(2)(t)), MaxPool(4)(t), ...]
            ps = HF.max_pool_pyramid(t, levels)
            return [sh(ps[0])] + ps[1:]

        N, _, H, W = x.shape
        cs = [HF.CatSlot(N, c, c, H >> i, W >> i, x) for i, c in enumerate((64, 128, 256, 512))]
        R1 = sh(self.c1(x, cs[0]))
        Q1 = pyr(R1, 4)
        R2 = sh(self.c2(Q1[0], cs[1]))
        Q2 = pyr(R2, 3)
        R3 = sh(self.c3(Q2[0], cs[2]))
        Q3 = pyr(R3, 2)
        R4 = sh(self.c4(Q3[0], cs[3]))
        Q4 = [sh(HF.max_pool2d(R4, 2))]
        R5 = self.c5(Q4[0])
        s64 = self.down64(R1, Q1)
        s128 = self.down128(R2, Q2)
        s256 = self.down256(R3, Q3)
        s512 = self.down512(R4, Q4)
        O1 = self.uc1(self.u1(HF.add_n(R5, s64[3], s128[2], s256[1], s512[0]), R4, cs[3]))
        O2 = self.uc2(self.u2(HF.add_n(O1, s64[2], s128[1], s256[0]), R3, cs[2]))
        O3 = self.uc3(self.u3(HF.add_n(O2, s64[1], s128[0]), R2, cs[1]))
        U4 = self.u4(HF.add_n(O3, s64[0]), R1, cs[0])
        del cs
        # --precision fp16 (configs[4]): the MLKA branch keeps bf16 16-bit operands (fp32 exponent
        # range).  Its InstanceNorms see input variances far below eps at the reference init, so
        # their backward multiplies gradients by up to ~1/sqrt(eps) per norm: under the fp16 mode's
        # loss scale (2^16) the branch's fp16 data-grads overflow while every other tensor stays
        # finite (tools/fp16_scale_probe.py; SURVEY.md §7 asks to keep this branch out of fp16).
        with HF.precision("bf16" if HF.get_precision() == "fp16" else None):
            Loc = self.local(x)
        # uc4(U4) + Loc: the block's shortcut GEMM adds Loc in its epilogue and the block sums into
        # Loc in place (no separate add of two 64 x 256^2 tensors)
        return HF.conv2d(self.uc4(U4, acc=Loc), self.res.weight, self.res.bias, stride=1, pad=1)
