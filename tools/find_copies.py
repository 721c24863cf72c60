"""List the torch-side tensor copies of one bench step (non-contiguous .contiguous(), dtype casts):
the call site, shape and bytes of each, to find residual torch kernels on the hot path."""
import os, sys, traceback, collections
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [REPO, os.path.join(REPO, "ds-gan_amd")]
import torch
from options.train_options import default_train_opt
from models import create_model
from oracle.recipe import synth_pair

torch.manual_seed(20)
m = create_model(default_train_opt(gpu_ids=[0], precision="bf16", batchSize=16))
A, B = synth_pair(16, 256, seed=0)
m.set_input({"A": A.cuda(), "B": B.cuda(), "A_paths": [""] * 16, "B_paths": [""] * 16})
m.optimize_parameters()
torch.cuda.synchronize()
hits = collections.Counter()
orig_cont, orig_float, orig_to = torch.Tensor.contiguous, torch.Tensor.float, torch.Tensor.to


def site():
    for fr in reversed(traceback.extract_stack()[:-2]):
        if "ds-gan_amd" in fr.filename or "models" in fr.filename:
            return "%s:%d" % (os.path.basename(fr.filename), fr.lineno)
    return "?"


def cont(self, *a, **k):
    if self.is_cuda and not self.is_contiguous(*a, **k):
        hits[("contiguous", site(), tuple(self.shape), self.numel() * self.element_size())] += 1
    return orig_cont(self, *a, **k)


def flt(self, *a, **k):
    if self.is_cuda and self.dtype != torch.float32:
        hits[("float", site(), tuple(self.shape), self.numel() * 4)] += 1
    return orig_float(self, *a, **k)


torch.Tensor.contiguous, torch.Tensor.float = cont, flt
m.optimize_parameters()
torch.cuda.synchronize()
torch.Tensor.contiguous, torch.Tensor.float = orig_cont, orig_float
for (kind, s, shape, nb), n in sorted(hits.items(), key=lambda kv: -kv[0][3] * kv[1]):
    print("%-10s %-28s %-24s %8.1f MB x%d" % (kind, s, shape, nb / 1e6, n))
