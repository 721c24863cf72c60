"""Which loss scale does the fp16 mode's backward tolerate?  One G+D step from the reference init
at the given size / batch for each power-of-two initial scale: whether the D and G backward
overflowed (the scaler skipped the step) and, without overflow, the largest |grad| of each
network (scaled).  python tools/fp16_scale_probe.py [size batch]"""
import os
import random
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]

import torch  # noqa: E402


def main():
    size = int(sys.argv[1]) if len(sys.argv) > 1 else 512
    batch = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    import dsgan_hip
    from oracle import dsgan_cpu as O
    from oracle.recipe import make_params, synth_pair
    from options.train_options import default_train_opt
    from models import create_model
    dsgan_hip.require_gpu()
    A, B = synth_pair(batch, size, seed=51)
    for e in (16, 14, 12, 10, 8, 6):
        random.seed(20)
        torch.manual_seed(20)
        m = create_model(default_train_opt(gpu_ids=[0], pool_size=0, precision="fp16", batchSize=batch, cuda_graph=0))
        with torch.no_grad():
            for net, pr in ((m.netG, make_params(O.g_param_spec(), "ref", 1000)),
                            (m.netD, make_params(O.d_param_spec(), "ref", 5000)),
                            (m.vgg, make_params(O.vgg_param_spec(True), "vgg", 7000))):
                for k, v in net.state_dict().items():
                    v.copy_(pr[k])
        for sc in (m.scaler_G, m.scaler_D):
            sc.state[0] = 2.0 ** e
        m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * batch, "B_paths": [""] * batch})
        m.optimize_parameters()
        torch.cuda.synchronize()
        gG, gD = m.flatG.grad, m.flatD.grad
        print("scale 2^%d: skipped G %s D %s  max|gG| %.3e  max|gD| %.3e  finite G %s" % (
            e, m.scaler_G.skipped_last(), m.scaler_D.skipped_last(), gG.abs().max().item(), gD.abs().max().item(),
            bool(torch.isfinite(gG).all())), flush=True)
        # the fp16 intermediate with the largest magnitude is what overflows: report per-parameter
        # tensors that are non-finite (first few, in backward order)
        names = {id(p): k for k, p in m.netG.named_parameters()}
        order = [names[id(p)] for p, _, _ in m.flatG.layout]          # backward order
        bad = [k for k in order if not torch.isfinite(dict(m.netG.named_parameters())[k].grad).all()]
        if bad:
            print("   non-finite G grads: %d of %d tensors; first in backward order: %s" % (
                len(bad), len(order), bad[:10]), flush=True)
            big = sorted(((dict(m.netG.named_parameters())[k].grad.abs().nan_to_num(0, 0, 0).max().item(), k)
                          for k in order if k not in bad), reverse=True)[:5]
            print("   largest finite G grads:", ["%s %.2e" % (k, v) for v, k in big], flush=True)
        del m
        torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
