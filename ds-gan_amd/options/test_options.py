"""Test flags (DSGAN/options/test_options.py:5-14), unchanged names and defaults."""
from .base_options import BaseOptions


class TestOptions(BaseOptions):
    def initialize(self, parser):
        parser = BaseOptions.initialize(self, parser)
        parser.add_argument("--ntest", type=int, default=float("inf"), help="# of test examples.")
        parser.add_argument("--results_dir", type=str, default="epoch_8_result_original/", help="saves results here.")
        parser.add_argument("--aspect_ratio", type=float, default=1.0, help="aspect ratio of result images")
        parser.add_argument("--phase", type=str, default="test_all/", help="train, val, test, etc")
        parser.add_argument("--which_epoch", type=str, default="1", help="which epoch to load?")
        parser.add_argument("--how_many", type=int, default=1000, help="how many test images to run")
        self.isTrain = False
        return parser


def default_test_opt(args=None, **overrides):
    """Programmatic TestOptions (``--model test`` unless overridden): the reference defaults
    plus ``overrides``; used by the inference tests."""
    import os
    o = TestOptions()
    opt = o.gather_options(["--model", "test"] + list(args or []))
    opt.isTrain = False
    opt.gpu_ids = [int(s) for s in str(opt.gpu_ids).split(",") if int(s) >= 0]
    opt.checkpoints_dir = os.path.join(os.environ.get("TMPDIR", "/tmp"), "dsgan_checkpoints")
    for k, v in overrides.items():
        setattr(opt, k, v)
    return opt
