"""train.py's per-iteration image metrics on the device (DSGAN/train.py:27-44, 110-124).

The reference moves image 0 of real_A / fake_B / real_B to the host every iteration, converts
them to uint8 and runs skimage SSIM / PSNR on the CPU.  ``TrainMetrics.update`` runs the same
arithmetic on the GPU (``dsgan_img_metrics``) and accumulates the sums in device memory; the
host reads them only when it prints (``averages``), so the loop has no per-iteration sync."""
import torch

from dsgan_hip._lib import call, ptr, stream


class TrainMetrics:
    def __init__(self, device):
        self.acc = torch.zeros(3, device=device, dtype=torch.float32)
        self.part = torch.empty(128, device=device, dtype=torch.float64)

    def reset(self):
        self.acc.zero_()

    def update(self, fake, real):
        """fake, real: one [C,H,W] image each in [-1, 1] (fake_B[0], real_B[0])."""
        fake, real = fake.detach().contiguous(), real.detach().contiguous()
        C, H, W = fake.shape
        call("dsgan_img_metrics", ptr(fake), ptr(real), C, H, W, ptr(self.part), ptr(self.acc), stream())

    def averages(self):
        s, p, n = self.acc.tolist()
        n = max(n, 1.0)
        return s / n, p / n
