"""G-forward-only inference model (DSGAN/models/test_model.py:5-42): ``--model test`` loads
netG from '{which_epoch}_net_G.pth' / '{which_epoch}_useSE_net_G.pth' and runs the generator's
HIP forward kernels under ``torch.no_grad()`` (BaseModel.test).  SURVEY.md §8 f-4."""
from dsgan_hip import functional as HF
from models import networks
from models.base_model import BaseModel


class TestModel(BaseModel):
    def name(self):
        return "TestModel"

    @staticmethod
    def modify_commandline_options(parser, is_train=True):
        assert not is_train, "TestModel cannot be used in train mode"
        parser.set_defaults(dataset_mode="single")
        parser.set_defaults(phase="test")
        parser.add_argument("--model_suffix", type=str, default="")
        return parser

    def initialize(self, opt):
        assert not opt.isTrain
        BaseModel.initialize(self, opt)
        if self.device.type != "cuda":
            raise RuntimeError("TestModel (MI355X build) needs a ROCm GPU: set --gpu_ids; "
                               "there is no CPU execution path")
        HF.set_precision(getattr(opt, "precision", "fp32"))
        self.loss_names = []
        self.visual_names = ["real_A", "fake_B"]
        self.model_names = ["G"]
        self.netG = networks.define_G(opt.input_nc, opt.output_nc, opt.ngf, opt.which_model_netG,
                                      opt.norm, not opt.no_dropout, opt.init_type, self.gpu_ids)

    def set_input(self, input):
        self.real_A = input["A"].to(self.device)
        self.image_paths = input["A_paths"]

    def forward(self):
        self.fake_B = self.netG(self.real_A)
