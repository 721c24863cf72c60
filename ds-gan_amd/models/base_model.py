"""BaseModel lifecycle (DSGAN/models/base_model.py:7-177) for the MI355X build.

Same public methods and semantics: initialize / setup / eval / test / set_input /
optimize_parameters / update_learning_rate / get_current_visuals / get_current_losses /
save_networks / load_networks / print_networks / set_requires_grad.  Device selection follows
``opt.gpu_ids`` as in the reference; with one process per GPU each rank owns ``cuda:LOCAL_RANK``.
"""
import os
from collections import OrderedDict

import torch

from . import networks


class BaseModel:
    @staticmethod
    def modify_commandline_options(parser, is_train):
        return parser

    def name(self):
        return "BaseModel"

    def initialize(self, opt):
        self.opt = opt
        self.gpu_ids = opt.gpu_ids
        self.isTrain = opt.isTrain
        self.device = torch.device("cuda:{}".format(self.gpu_ids[0])) if self.gpu_ids else torch.device("cpu")
        self.save_dir = os.path.join(opt.checkpoints_dir, opt.name)
        self.loss_names = []
        self.model_names = []
        self.visual_names = []
        self.image_paths = []

    def set_input(self, input):
        self.input = input

    def forward(self):
        pass

    def setup(self, opt, parser=None):
        if self.isTrain:
            self.schedulers = [networks.get_scheduler(optimizer, opt) for optimizer in self.optimizers]
        if not self.isTrain or opt.continue_train:
            self.load_networks(opt.which_epoch)
        self.print_networks(opt.verbose)

    def eval(self):
        for name in self.model_names:
            if isinstance(name, str):
                getattr(self, "net" + name).eval()

    def test(self):
        with torch.no_grad():
            self.forward()

    def get_image_paths(self):
        return self.image_paths

    def optimize_parameters(self):
        pass

    def update_learning_rate(self):
        for scheduler in self.schedulers:
            scheduler.step()
        lr = self.optimizers[0].param_groups[0]["lr"]
        print("learning rate = %.7f" % lr)

    def get_current_visuals(self):
        visual_ret = OrderedDict()
        for name in self.visual_names:
            if isinstance(name, str):
                visual_ret[name] = getattr(self, name)
        return visual_ret

    def get_current_losses(self):
        errors_ret = OrderedDict()
        for name in self.loss_names:
            if isinstance(name, str):
                v = getattr(self, "loss_" + name)
                errors_ret[name] = float(v.detach() if torch.is_tensor(v) else v)
        return errors_ret

    def save_networks(self, which_epoch):
        """'{epoch}_useSE_net_{G,D}.pth' as the reference writes (:95).  Keys carry no
        ``module.`` prefix (no DataParallel wrapper); load_networks accepts both."""
        os.makedirs(self.save_dir, exist_ok=True)
        for name in self.model_names:
            if isinstance(name, str):
                save_filename = "%s_useSE_net_%s.pth" % (which_epoch, name)
                net = getattr(self, "net" + name)
                sd = OrderedDict((k, v.detach().cpu().clone()) for k, v in net.state_dict().items())
                torch.save(sd, os.path.join(self.save_dir, save_filename))

    def load_networks(self, which_epoch):
        """Reads '{epoch}_net_{name}.pth' like the reference (:119) and, if that is absent, the
        '{epoch}_useSE_net_{name}.pth' this build (and the reference) saves -- the reference's
        save/load name mismatch is bridged instead of failing.  ``module.`` prefixes from
        DataParallel checkpoints are stripped.  As the reference's ``load_state_dict(strict=False)``
        (:148): missing / unexpected keys are allowed (and printed), a shape mismatch raises."""
        for name in self.model_names:
            if isinstance(name, str):
                net = getattr(self, "net" + name)
                cands = ["%s_net_%s.pth" % (which_epoch, name), "%s_useSE_net_%s.pth" % (which_epoch, name)]
                paths = [os.path.join(self.save_dir, c) for c in cands]
                path = next((p for p in paths if os.path.exists(p)), paths[0])
                print("loading the model from %s" % path)
                state_dict = torch.load(path, map_location="cpu", weights_only=True)
                state_dict = OrderedDict((k[7:] if k.startswith("module.") else k, v) for k, v in state_dict.items())
                state_dict = {k: v for k, v in state_dict.items()
                              if not (k.endswith("running_mean") or k.endswith("running_var"))}
                own = net.state_dict()
                bad = ["%s: checkpoint %s vs model %s" % (k, tuple(v.shape), tuple(own[k].shape))
                       for k, v in state_dict.items() if k in own and own[k].shape != v.shape]
                if bad:
                    raise RuntimeError("Error(s) in loading state_dict for %s:\n\tsize mismatch for %s"
                                       % (type(net).__name__, "\n\tsize mismatch for ".join(bad)))
                missing = [k for k in own if k not in state_dict]
                unexpected = [k for k in state_dict if k not in own]
                if missing or unexpected:
                    print("load_networks(%s): missing keys %s, unexpected keys %s" % (name, missing, unexpected))
                with torch.no_grad():
                    for k, v in state_dict.items():
                        if k in own:
                            own[k].copy_(v.to(own[k].device, own[k].dtype))

    def print_networks(self, verbose):
        print("---------- Networks initialized -------------")
        for name in self.model_names:
            if isinstance(name, str):
                net = getattr(self, "net" + name)
                num_params = sum(p.numel() for p in net.parameters())
                if verbose:
                    print(net)
                print("[Network %s] Total number of parameters : %.3f M" % (name, num_params / 1e6))
        print("-----------------------------------------------")

    def set_requires_grad(self, nets, requires_grad=False):
        if not isinstance(nets, list):
            nets = [nets]
        for net in nets:
            if net is not None:
                for param in net.parameters():
                    param.requires_grad = requires_grad
