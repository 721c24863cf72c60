"""The DS-GAN train step (DSGAN/models/pix2pix_model.py), MI355X-native.

``--model pix2pix`` resolves here through the same registry rule as the reference, and the
class keeps the reference's API: ``initialize / set_input / forward / backward_D /
backward_G / optimize_parameters / get_img_tir / get_img_gen / get_img_label`` plus the
``loss_*`` / ``real_A`` / ``fake_B`` / ``real_B`` / ``netG`` / ``netD`` / ``optimizers``
attributes that ``train.py`` reads.

What runs underneath: every forward/backward op is a fused HIP kernel (``dsgan_hip``), params
and grads of each network live in one flat buffer updated by one fused-Adam launch, and under
``torchrun`` the two gradient exchanges are RCCL all-reduces (``dsgan_hip.dist``).

Deliberate, documented deviations:
  * q1: untyped loss-weight flags are cast to numbers (the reference crashes on CLI values);
  * multi-GPU (one process per GPU): each rank holds its chunk of the global batch (data/), so
    the gradients are made equal to the reference's global-batch gradient
    (nn.DataParallel computes every loss on the gathered batch, networks.py:74-77): the batch
    *means* (BCE, L1, VGG-L1, SSIM) are weighted by world * n_rank / n_global (1 when the global
    batch divides evenly), the TV term -- a batch *sum*, :189-191 -- by the world size, and the
    gradients are averaged; the ImagePool is per rank (its python RNG seeded 20 + 1000 * rank);
  * the unused VGG relu5_3 block is not computed (the loss never reads it, :182-186);
  * --precision fp16 (BASELINE configs[4]): both backward passes run on a dynamically scaled loss
    (dsgan_hip.amp.LossScaler, GradScaler semantics on the device), the optimizers unscale, and
    an overflowed step is skipped; the logged losses are the unscaled ones;
  * --nonfinite_guard (on by default in bf16): the same device-side check with a unit scale -- an
    optimizer step whose flat gradient holds inf/nan is skipped (the reference would write NaN
    into its weights and never recover); with finite gradients nothing changes.
"""
import os
import random

import torch

from dsgan_hip import _lib
from dsgan_hip import functional as HF
from dsgan_hip import dist as hdist
from dsgan_hip.flat import FlatParams, FlatAdam
from dsgan_hip.amp import LossScaler
from util.image_pool import ImagePool
from .base_model import BaseModel
from . import networks

# backward_D runs D once on the fake and real batches stacked (DSGAN_D_BATCH=0: two passes, as the
# reference's code reads: DSGAN/models/pix2pix_model.py:141-160); same logits, the weight-grads to fp32
# reassociation (tests/test_dbatch_gpu.py).  (Round 5 had it off in fp16 after a configs[4] run drifted:
# the cause was a NaN in the SSIM backward, not the stacked pass -- losses.hip ssim_fwd_kernel.)
D_BATCH = os.environ.get("DSGAN_D_BATCH", "1") != "0"

# The G step's perceptual forward (VGG16 over fake_B and its four L1s) depends only on the generator's
# output, not on the D step: it runs on the VGG side stream while the D step runs on the main stream,
# and the G step joins the side stream before it reads the loss (DSGAN_VGG_OVERLAP=0: in program
# order, as the reference's code reads: DSGAN/models/pix2pix_model.py:164-199).  The autograd node is
# created on the main stream, so its backward (the VGG data-grad chain) stays there.
VGG_OVERLAP = os.environ.get("DSGAN_VGG_OVERLAP", "1") != "0"


class GraphCaptureError(RuntimeError):
    """Under DDP, graph B's capture (the step with its RCCL exchanges) failed: not recoverable by
    an eager fallback, the run ends."""


class _CaptureDeclined(RuntimeError):
    """Graph A's capture failed on some rank; every rank raises this together (one agreement)."""


def _fusable(*xs):
    """Loss terms HF.loss_sum takes: 0-d fp32 device tensors (a disabled term may be a python 0)."""
    ts = [x for x in xs if not (not torch.is_tensor(x) and x == 0)]
    return bool(ts) and len(ts) <= 8 and all(torch.is_tensor(x) and x.dim() == 0 and x.dtype == torch.float32
                                             and x.is_cuda for x in ts)
from .vgg import Vgg16

POOL_SEED = 20   # DSGAN/train.py:48 setup_seed(20): the ImagePool's RNG on ranks > 0 is offset from it


class Pix2PixModel(BaseModel):
    def name(self):
        return "Pix2PixModel"

    @staticmethod
    def modify_commandline_options(parser, is_train=True):
        if is_train:
            parser.add_argument("--lambda_L1", type=float, default=100.0, help="weight for L1 loss")
        return parser

    def initialize(self, opt):
        BaseModel.initialize(self, opt)
        if self.device.type != "cuda":
            raise RuntimeError("Pix2PixModel (MI355X build) needs a ROCm GPU: set --gpu_ids; "
                               "there is no CPU execution path")
        HF.set_precision(getattr(opt, "precision", "fp32"))
        self.isTrain = opt.isTrain
        self.loss_names = ["G_GAN", "G_L1", "D_real", "D_fake"]
        self.visual_names = ["real_A", "fake_B", "real_B"]
        self.model_names = ["G", "D"] if self.isTrain else ["G"]
        self.use_gan = int(opt.use_GAN)
        self.w_vgg = float(opt.w_vgg)
        self.w_tv = float(opt.w_tv)
        self.w_gan = float(opt.w_gan)
        self.w_ss = float(opt.w_ss)
        self.use_condition = int(opt.use_condition)
        self.ssim_kind = getattr(opt, "ssim_loss", "ssim")
        self.netG = networks.define_G(opt.input_nc, opt.output_nc, opt.ngf, opt.which_model_netG,
                                      opt.norm, not opt.no_dropout, opt.init_type, self.gpu_ids)
        if self.isTrain:
            use_sigmoid = opt.no_lsgan
            d_in = opt.input_nc + opt.output_nc if self.use_condition == 1 else opt.input_nc
            self.netD = networks.define_D(d_in, opt.ndf, opt.which_model_netD, opt.n_layers_D,
                                          opt.norm, use_sigmoid, opt.init_type, self.gpu_ids)
        if self.isTrain:
            W, r = hdist.world_size(), hdist.rank()
            # one process: the global python `random`, consumed exactly as the reference does
            self.fake_AB_pool = ImagePool(opt.pool_size, rng=None if W == 1 else random.Random(POOL_SEED + 1000 * r))
            self.criterionGAN = networks.GANLoss(use_lsgan=opt.no_lsgan).to(self.device)
            self.criterionL1 = HF.l1_loss
            self.vgg = Vgg16(getattr(opt, "vgg_weights", "") or None).to(self.device)
            # flat param/grad buffers + fused Adam (one launch per network per step)
            order = self.netG.backward_order() if hasattr(self.netG, "backward_order") else None
            self.flatG = FlatParams(self.netG, self.device, order=order)
            self.flatD = FlatParams(self.netD, self.device)
            # the two exchanges run whenever there is more than one rank (``exchange`` can force
            # them on a 1-rank group: the RCCL stream-ordering test of tests/test_ddp_gpu.py)
            self.exchange = W > 1
            self.g_buckets = hdist.GradBuckets(self.flatG.grad, self.flatG.layout) if W > 1 else None
            hdist.broadcast_params(self.flatG)
            hdist.broadcast_params(self.flatD)
            self.optimizers = []
            fp16 = HF.get_precision() == "fp16"
            guard = int(getattr(opt, "nonfinite_guard", -1))
            guard = HF.get_precision() == "bf16" if guard < 0 else bool(guard)
            if fp16:
                self.scaler_G, self.scaler_D = LossScaler(self.device), LossScaler(self.device)
            elif guard:   # unit-scale scalers: the inf/nan check + skip only
                self.scaler_G, self.scaler_D = LossScaler.guard(self.device), LossScaler.guard(self.device)
            else:
                self.scaler_G = self.scaler_D = None
            self.optimizer_G = FlatAdam(self.flatG, lr=opt.lr, betas=(opt.beta1, 0.999), scaler=self.scaler_G)
            self.optimizer_D = FlatAdam(self.flatD, lr=opt.lr, betas=(opt.beta1, 0.999), scaler=self.scaler_D)
            self.optimizers.append(self.optimizer_G)
            self.optimizers.append(self.optimizer_D)
            self.tv_scale = float(W)
            self.mean_w = 1.0   # world * n_rank / n_global, set per batch by set_input
            self._vgg_stream = torch.cuda.Stream(self.device)
            self._real_feats = None
            self._feats_joined = False
            # the step as two captured HIP graphs (see _graph_step): optimizer step counts on the
            # device (the fp16 scalers or the bf16 guard); under DDP the RCCL exchanges are captured
            # into the second graph, so the process group must be RCCL ("nccl"), not gloo
            cg = int(getattr(opt, "cuda_graph", -1))
            can = self.scaler_G is not None and (W == 1 or hdist.backend() == "nccl")
            if cg == 1 and not can:
                raise ValueError("--cuda_graph 1 needs device-side step counts (--precision fp16, or bf16 "
                                 "with the non-finite guard) and, under DDP, the RCCL backend")
            self.cuda_graph = can and cg != 0
            self._graphs = {}          # (input shapes, mean_w) -> one captured graph pair (_capture)
            self._graph_warm = set()   # the keys whose eager warm-up step has run
            # optimizer-step calls per network: host counters, since a graph replay never enters
            # FlatAdam.step (the scalers count the applied steps on the device)
            self.step_calls = {"G": 0, "D": 0}
            # backward_D's stacked batch-2N D pass (D_BATCH); an attribute so tests can compare the two forms
            self.d_batch = D_BATCH
            self.vgg_overlap = VGG_OVERLAP
            self._pre_perc = None

    def set_input(self, input):
        AtoB = self.opt.which_direction == "AtoB"
        A = input["A" if AtoB else "B"].to(self.device, non_blocking=True)
        B = input["B" if AtoB else "A"].to(self.device, non_blocking=True)
        self.image_paths = input["A_paths" if AtoB else "B_paths"]
        if self.isTrain:
            W = hdist.world_size()
            n = int(A.shape[0])
            self.mean_w = float(W * n) / float(input.get("global_batch", W * n))
            ent = self._graphs.get(self._graph_key(A, B, self.mean_w))
            if ent is not None:   # a captured graph pair reads its static input buffers
                ent["vars"]["real_A"].copy_(A, non_blocking=True)
                ent["vars"]["real_B"].copy_(B, non_blocking=True)
                A, B = ent["vars"]["real_A"], ent["vars"]["real_B"]
        self.real_A, self.real_B = A, B

    def forward(self):
        self.fake_B = self.netG(self.real_A)

    def backward_D(self, fake_AB=None):
        if fake_AB is not None:   # (the graph step: the pool's output, queried between the two graphs)
            pass
        elif self.use_condition == 1:
            fake_AB = self.fake_AB_pool.query(HF.cat_channels(self.real_A, self.fake_B.detach()))
        else:
            fake_AB = self.fake_B
        fake_AB = fake_AB.detach()
        if self.d_batch and fake_AB.dim() == 4 and fake_AB.dtype == torch.float32:
            # the fake and real passes as ONE batch-2N pass of D (D's ops are per-sample: the same
            # outputs, half the launches); neither half needs an input grad
            N, C, H, W = fake_AB.shape
            AB = torch.empty((2 * N, C, H, W), device=fake_AB.device, dtype=torch.float32)
            HF.copy_into(AB[:N], fake_AB)
            if self.use_condition == 1:
                Ca = self.real_A.shape[1]
                HF.copy_into(AB[N:, :Ca], self.real_A)
                HF.copy_into(AB[N:, Ca:], self.real_B)
            else:
                HF.copy_into(AB[N:], self.real_B)
            pred = self.netD(AB)
            pred_fake, pred_real = pred[:N], pred[N:]
        else:
            pred_fake = self.netD(fake_AB)
            real_AB = HF.cat_channels(self.real_A, self.real_B) if self.use_condition == 1 else self.real_B
            pred_real = self.netD(real_AB)
        self.pred_fake, self.pred_real = pred_fake, pred_real
        self.loss_D_fake = self.criterionGAN(pred_fake, False)
        self.loss_D_real = self.criterionGAN(pred_real, True)
        if _fusable(self.loss_D_fake, self.loss_D_real):   # one launch each way (HF.loss_sum)
            self.loss_D = HF.loss_sum([(self.loss_D_fake, 1.0), (self.loss_D_real, 1.0)], 0.5)
        else:
            self.loss_D = (self.loss_D_fake + self.loss_D_real) * 0.5
        loss = self.loss_D if self.mean_w == 1.0 else self.loss_D * self.mean_w
        with HF.deferred_splits():   # the weight-grads' split reductions: one batched flush at the end
            (loss if self.scaler_D is None else self.scaler_D.scale(loss)).backward()

    def backward_G(self):
        if self.use_gan == 1:
            fake_AB = HF.cat_channels(self.real_A, self.fake_B) if self.use_condition == 1 else self.fake_B
            self.loss_G_GAN = self.criterionGAN(self.netD(fake_AB), True)
        else:
            self.loss_G_GAN = 0
        # the four image losses sum their fake_B grads in one buffer (HF.share: the L1 / TV / SSIM
        # backward kernels accumulate in place) instead of through autograd adds; same order of sums
        pre, self._pre_perc = self._pre_perc, None
        if pre is not None:   # the perceptual forward already ran on the side stream (VGG_OVERLAP)
            fB, self.real_B_features, self.loss_vgg = pre
            self.loss_G_L1 = self.criterionL1(fB, self.real_B)
            torch.cuda.current_stream(self.device).wait_stream(self._vgg_stream)
        else:
            fB = HF.share(self.fake_B)
            self.loss_G_L1 = self.criterionL1(fB, self.real_B)
            self.real_B_features = self._take_real_features()
            # L1(f1,r1) + L1(f2,r2) + L1(f3,r3) + L1(f0,r0) over vgg(fake_B): one fused node whose
            # backward is the hand-written VGG data-grad chain (vgg.py / functional.PerceptualL1Fn)
            self.loss_vgg = self.vgg.perceptual_l1(fB, self.real_B_features)
        self.tv_loss = HF.tv_loss(fB, self.tv_scale / (320 * 256))
        # 1 - ssim((real_B+1)/2, (fake_B+1)/2, data_range=1): the affine map is fused in-kernel
        # (--ssim_loss ms_ssim: the 5-level MS-SSIM of DSGAN/MS_SSIM.py:153-225 instead)
        if self.ssim_kind == "ms_ssim":
            self._ssim_val = HF.ms_ssim_loss_affine(self.real_B, fB, 0.5, 0.5, 1.0)
        else:
            self._ssim_val = HF.ssim_affine(self.real_B, fB, 0.5, 0.5, 1.0)
        if self.mean_w == 1.0 and _fusable(self.loss_G_GAN, self.loss_G_L1, self.loss_vgg, self.tv_loss, self._ssim_val):
            # the same sum in one launch each way: w_ss * (1 - ssim) is the (w_ss, 1, -1) term
            self.loss_G = HF.loss_sum([(self.loss_G_GAN, self.w_gan), (self.loss_G_L1, 1.0),
                                       (self.loss_vgg, self.w_vgg), (self.tv_loss, self.w_tv),
                                       (self._ssim_val, self.w_ss, 1.0, -1.0)])
        else:
            self.loss_G = (self.loss_G_GAN * self.w_gan + self.loss_G_L1 + self.loss_vgg * self.w_vgg
                           + self.tv_loss * self.w_tv + self.w_ss * self.loss_ssim)
        if self.mean_w == 1.0:
            loss = self.loss_G
        else:   # ragged global batch under DDP: reweight the batch means, not the TV sum
            loss = ((self.loss_G_GAN * self.w_gan + self.loss_G_L1 + self.loss_vgg * self.w_vgg + self.w_ss * self.loss_ssim)
                    * self.mean_w + self.tv_loss * self.w_tv)
        with HF.deferred_splits():
            (loss if self.scaler_G is None else self.scaler_G.scale(loss)).backward()

    @property
    def loss_ssim(self):
        """1 - ssim (the logged term; the step's loss_sum folds it into its (w_ss, 1, -1) term)."""
        return 1 - self._ssim_val

    def _launch_real_features(self):
        """vgg(real_B) (frozen, no grad) depends only on the input: run it on a side stream so it
        overlaps the generator forward and the D step; backward_G joins the stream."""
        main = torch.cuda.current_stream(self.device)
        side = self._vgg_stream
        side.wait_stream(main)
        with torch.cuda.stream(side):
            self.real_B.record_stream(side)
            feats = self.vgg.loss_features(self.real_B)
        for f in feats:
            f.record_stream(main)
        self._real_feats = feats

    def _launch_fake_perceptual(self):
        """The G step's perceptual forward on the VGG side stream, ahead of the D step (VGG_OVERLAP):
        it follows the real-feature pass on that stream, so it needs no join of its own; backward_G
        joins the stream before reading the loss."""
        if self._real_feats is None:
            self._launch_real_features()
        feats, self._real_feats = self._real_feats, None
        fB = HF.share(self.fake_B)
        loss = self.vgg.perceptual_l1(fB, feats, side=self._vgg_stream)
        self._pre_perc = (fB, feats, loss)

    def _take_real_features(self):
        if self._real_feats is None:
            self._launch_real_features()
        if not self._feats_joined:   # (the graph step joined the side stream inside its first graph)
            torch.cuda.current_stream(self.device).wait_stream(self._vgg_stream)
        feats, self._real_feats = self._real_feats, None
        return feats

    def nonfinite_report(self):
        """{'G': (skipped, calls), 'D': (skipped, calls)}: optimizer steps the non-finite guard (or
        the fp16 loss scaler) skipped so far, out of the steps called.  Empty without scalers.
        Reads the scalers' device state, so it synchronises: call it at logging time only."""
        out = {}
        for net, sc in (("G", self.scaler_G), ("D", self.scaler_D)):
            if sc is not None:
                n = self.step_calls[net]
                out[net] = (n - sc.applied_steps(), n)
        return out

    def optimize_parameters(self):
        self.step_calls["G"] += 1
        if self.use_gan == 1:
            self.step_calls["D"] += 1
        if self.cuda_graph:
            return self._graph_step()
        self._eager_step()

    def _eager_step(self):
        self._launch_real_features()
        self.forward()
        self._d_and_g_steps()

    # ---- the step as two HIP graphs ----
    # ~760 kernel launches per step leave ~1 ms/step of dispatch gaps between them.  Replayed from
    # graphs they go back to back.  The ImagePool query draws python `random` per image
    # (DSGAN/util/image_pool.py:17-31), so the step is split around it: graph A = the VGG16
    # real-feature pass (side stream, joined inside A) + G forward + cat(real_A, fake_B); the pool
    # query runs eagerly into a static buffer (the same draws, in the same order, as the reference);
    # graph B = the D step and the G step (backward, scaler checks, both Adams) and, under DDP, the
    # RCCL exchanges: the D all-reduce before optimizer_D.step() and the G buckets, started from the
    # autograd thread as their weight-grads are launched, exactly as in the eager step -- captured,
    # they replay on RCCL's stream with the same dependencies (every rank captures the same
    # collectives in the same order, as the eager step already requires).
    # Everything a replay needs from the host is fixed at capture: shapes, loss weights, the
    # learning rates and the Adam step counts (device-side under the scalers / guard).  One graph
    # pair is kept per input shape and loss weight (with one process a ragged last batch gets its
    # own, captured once, after one eager warm-up step of that shape); a learning-rate change
    # re-captures that shape's pair.
    @staticmethod
    def _graph_key(A, B, mean_w):
        return (tuple(A.shape), tuple(B.shape), mean_w)

    def _graph_step(self):
        if self.mean_w != 1.0 and hdist.world_size() > 1:
            # a ragged global batch under DDP: the ranks' chunks differ in size, so their graph keys
            # would too, and the capture / replay decisions (with the capture's one agreement
            # all-reduce) must be the same on every rank -- those steps run eager.  mean_w is 1 on
            # every rank or on none (W * n == the global batch only when all chunks are equal).
            return self._eager_step()
        key = self._graph_key(self.real_A, self.real_B, self.mean_w)
        lrs = tuple(float(o.param_groups[0]["lr"]) for o in self.optimizers)
        ent = self._graphs.get(key)
        if ent is not None and ent["lr"] != lrs:
            # a learning-rate change: re-capture (set_input copied the inputs into this pair's static
            # buffers, which real_A / real_B point at; _capture clones them)
            del self._graphs[key]
            ent = None
        if ent is None:
            if key not in self._graph_warm:   # one eager step first (lazy allocations, cached weight copies)
                self._graph_warm.add(key)
                return self._eager_step()
            err = None
            try:
                ent = self._capture(lrs)
            except GraphCaptureError:   # DDP: graph B's capture failed after collectives were recorded
                raise
            except Exception as e:   # noqa: BLE001 -- a capture failure must not end the run: eager from here on
                err = e
            if err is not None:
                # one process, or every rank declined graph A together (_capture's agreement): the
                # invalidated capture's error is still pending in the HIP runtime
                _lib.load().dsgan_clear_launch_error()
                print("[Pix2PixModel] HIP graph capture failed (%r): running the eager step" % (err,))
                self._graphs, self.cuda_graph, self._feats_joined = {}, False, False
                HF.GRAD_READY[0] = None
                torch.cuda.synchronize(self.device)
                return self._eager_step()
            self._graphs[key] = ent
        self.__dict__.update(ent["vars"])   # this pair's outputs / losses / static inputs
        ent["gA"].replay()
        if self.use_gan == 1 and self.use_condition == 1:
            self.fake_AB_pool.query(self._cat_fake, out=self._fake_AB_buf)
        ent["gB"].replay()

    def _capture(self, lrs):
        """Capture this shape's graph pair.  Graph A (VGG real features, G forward) holds no
        collective: if its capture fails on any rank, every rank learns it from one MIN all-reduce
        and raises _CaptureDeclined together (the caller runs eager from then on, the ranks still in
        step).  Graph B holds the RCCL exchanges: a rank whose capture of B fails may have recorded a
        different sequence of collectives than the others, so under DDP that ends the run
        (GraphCaptureError) instead of an eager fallback whose collectives could pair up wrongly."""
        self.real_A, self.real_B = self.real_A.clone(), self.real_B.clone()   # the static inputs
        torch.cuda.synchronize(self.device)
        pool = torch.cuda.graph_pool_handle()
        gA, gB = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
        cond = self.use_gan == 1 and self.use_condition == 1
        # thread_local capture mode: the RCCL process group's watchdog thread polls the events of
        # earlier (eager) collectives; in the default global mode such a query from another thread
        # invalidates the capture.  The capturing thread itself still may not make unsafe calls.
        err_a = None
        try:
            with torch.cuda.graph(gA, pool=pool, capture_error_mode="thread_local"):
                try:
                    self._launch_real_features()
                    self.forward()
                    if cond:
                        self._cat_fake = HF.cat_channels(self.real_A, self.fake_B.detach())
                        self._fake_AB_buf = torch.empty_like(self._cat_fake)
                finally:
                    # the VGG side stream joins the capture stream even when the forward raised: an
                    # unjoined forked stream makes the capture's end fail and leaves the capture
                    # stream current (and capturing) for the eager step that follows
                    torch.cuda.current_stream(self.device).wait_stream(self._vgg_stream)
                self._feats_joined = True
        except Exception as e:   # noqa: BLE001 -- agreed on below, before anything is re-raised
            err_a = e
            _lib.load().dsgan_clear_launch_error()
            self._feats_joined = False
        if not hdist.all_ranks_true(err_a is None, self.device):   # every rank captures B, or none does
            raise _CaptureDeclined(err_a if err_a is not None else "graph A capture failed on another rank")
        try:
            with torch.cuda.graph(gB, pool=pool, capture_error_mode="thread_local"):
                self._d_and_g_steps(self._fake_AB_buf if cond else None)
        except Exception as e:
            if hdist.world_size() > 1:
                raise GraphCaptureError("HIP graph capture of the D / G step (with its RCCL exchanges) failed on "
                                        "rank %d: %r -- ending the run (the ranks' recorded collectives may "
                                        "differ)" % (hdist.rank(), e)) from e
            raise
        finally:
            self._feats_joined = False
            HF.GRAD_READY[0] = None
        # every tensor attribute the captured step left on the model (static inputs, fake_B, the
        # losses, ...): restored before each replay of this pair
        tvars = {k: v for k, v in self.__dict__.items() if torch.is_tensor(v)}
        return {"gA": gA, "gB": gB, "lr": lrs, "vars": tvars}

    def _d_and_g_steps(self, fake_AB=None):
        if self.vgg_overlap and self.use_gan == 1:
            self._launch_fake_perceptual()
        if self.use_gan == 1:
            self.set_requires_grad(self.netD, True)
            self.optimizer_D.zero_grad()
            self.backward_D(fake_AB)
            if self.exchange:
                hdist.allreduce_mean_(self.flatD.grad, force=True)
            if self.scaler_D is not None:
                self.scaler_D.check(self.flatD.grad)
            self.optimizer_D.step()
        else:
            self.loss_D_fake = 0
            self.loss_D_real = 0
        self.set_requires_grad(self.netD, False)
        self.optimizer_G.zero_grad()
        if self.g_buckets is not None:
            self.g_buckets.arm()       # G grad buckets all-reduce as backward_G fills them
        self.backward_G()
        if self.g_buckets is not None:
            self.g_buckets.finish()
        if self.scaler_G is not None:
            self.scaler_G.check(self.flatG.grad)
        self.optimizer_G.step()

    # ---- train.py helpers (DSGAN/models/pix2pix_model.py:292-310) ----
    def get_img_tir(self, input):
        self.real_A = input["A"].to(self.device)
        return ((self.real_A + 1) / 2) * 255

    def get_img_gen(self, input):
        AtoB = self.opt.which_direction == "AtoB"
        self.real_B = input["B" if AtoB else "A"].to(self.device)
        self.fake_B = self.netG(self.real_A)
        return ((self.fake_B + 1) / 2) * 255

    def get_img_label(self, input):
        AtoB = self.opt.which_direction == "AtoB"
        self.real_B = input["B" if AtoB else "A"].to(self.device)
        return ((self.real_B + 1) / 2) * 255

    def get_img_nir(self, input):
        AtoB = self.opt.which_direction == "AtoB"
        self.real_A = input["A" if AtoB else "B"].to(self.device)
        return ((self.real_A + 1) / 2) * 255
