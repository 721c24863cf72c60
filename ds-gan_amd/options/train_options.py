"""Training flags (DSGAN/options/train_options.py:5-27), unchanged names and defaults."""
from .base_options import BaseOptions


class TrainOptions(BaseOptions):
    def initialize(self, parser):
        parser = BaseOptions.initialize(self, parser)
        parser.add_argument("--display_freq", type=int, default=100, help="frequency of showing training results on screen")
        parser.add_argument("--display_ncols", type=int, default=4, help="images per row in the web display")
        parser.add_argument("--update_html_freq", type=int, default=1000, help="frequency of saving training results to html")
        parser.add_argument("--print_freq", type=int, default=100, help="frequency of showing training results on console")
        parser.add_argument("--save_latest_freq", type=int, default=5000, help="frequency of saving the latest results")
        parser.add_argument("--save_epoch_freq", type=int, default=50, help="frequency of saving checkpoints at the end of epochs")
        parser.add_argument("--continue_train", action="store_true", default=False, help="continue training: load the latest model")
        parser.add_argument("--epoch_count", type=int, default=1, help="the starting epoch count")
        parser.add_argument("--phase", type=str, default="train_all/", help="train, val, test, etc")
        parser.add_argument("--which_epoch", type=str, default="1", help="which epoch to load?")
        parser.add_argument("--niter", type=int, default=10, help="# of iter at starting learning rate")
        parser.add_argument("--niter_decay", type=int, default=10, help="# of iter to linearly decay learning rate to zero")
        parser.add_argument("--beta1", type=float, default=0.5, help="momentum term of adam")
        parser.add_argument("--lr", type=float, default=0.0002, help="initial learning rate for adam")
        parser.add_argument("--no_lsgan", action="store_true", help="do *not* use least square GAN, if false, use vanilla GAN")
        parser.add_argument("--pool_size", type=int, default=50, help="the size of image buffer that stores previously generated images")
        parser.add_argument("--no_html", action="store_true", help="do not save intermediate training results")
        parser.add_argument("--lr_policy", type=str, default="lambda", help="learning rate policy: lambda|step|plateau")
        parser.add_argument("--lr_decay_iters", type=int, default=50, help="multiply by a gamma every lr_decay_iters iterations")
        # build extension (not a reference flag): the structural term of backward_G
        # (DSGAN/models/pix2pix_model.py:193-195 uses single-scale ssim; BASELINE config 4 names the
        # gaussian-pyramid MS-SSIM of DSGAN/MS_SSIM.py:153-225, which needs images > 160 px)
        parser.add_argument("--ssim_loss", type=str, default="ssim", choices=["ssim", "ms_ssim"],
                            help="structural loss term: ssim (reference) or ms_ssim (opt-in)")
        # build extension: a device-side inf/nan scan of each network's flat gradient before its Adam
        # step; a non-finite gradient skips that optimizer step (parameters and moments untouched)
        # instead of writing NaN into the weights.  -1 = on for --precision bf16 (fp16 always has it
        # through its loss scaler), off for the fp32 parity mode.
        parser.add_argument("--cuda_graph", type=int, default=-1, choices=[-1, 0, 1],
                            help="replay optimize_parameters as two captured HIP graphs around the ImagePool "
                                 "query (-1: on for one process with device-side loss scaling / guard)")
        parser.add_argument("--nonfinite_guard", type=int, default=-1, choices=[-1, 0, 1],
                            help="skip an optimizer step whose gradient has inf/nan (-1: on for bf16)")
        self.isTrain = True
        return parser


def default_train_opt(args=None, **overrides):
    """Programmatic TrainOptions (no argv, no opt.txt written): the reference defaults plus
    ``overrides``.  Used by bench.py, __graft_entry__.smoke() and the tests."""
    import os
    o = TrainOptions()
    opt = o.gather_options(list(args or []))
    opt.isTrain = True
    opt.gpu_ids = [int(s) for s in str(opt.gpu_ids).split(",") if int(s) >= 0]
    if "LOCAL_RANK" in os.environ and opt.gpu_ids:
        opt.gpu_ids = [int(os.environ["LOCAL_RANK"])]
    opt.checkpoints_dir = os.path.join(os.environ.get("TMPDIR", "/tmp"), "dsgan_checkpoints")
    for k, v in overrides.items():
        setattr(opt, k, v)
    return opt
