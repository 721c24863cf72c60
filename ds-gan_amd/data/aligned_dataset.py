"""Paired TIR/RGB dataset (DSGAN/data/aligned_dataset.py:27-90) with the transforms on the GPU.

The host side decodes (PIL ``.convert('RGB')``), draws the crop offsets and the flip with
python ``random`` in the reference's order (w_offset, h_offset, then ``random.random() < 0.5``
unless --no_flip, :61-62, :74) and crops the uint8 image.  ToTensor / Normalize(0.5, 0.5) /
flip / RGB->gray then run as one HIP kernel on the uploaded uint8 batch (``dsgan_u8_to_image``,
bit-exact with the torch CPU ops), so a batch crosses PCIe as uint8 (4x fewer bytes).

Seeded data order is parity-PINNED only for serial, unshuffled loading (nThreads=0,
serial_batches; tests/test_eval_gpu.py checks that path bit-exactly).  With worker processes
(nThreads > 0) each worker's ``random`` is reseeded from torch's CPU base seed, and shuffling
draws from the torch CPU generator, whose state after create_model differs from the
reference's: torchvision's vgg16() also initialises its classifier from the global generator,
which this build (conv holders only, ImageNet weights or a private-generator init) does not.
So under seed 20 the shuffled order and the crop/flip draws are valid but parity-UNPINNED."""
import os
import random

import numpy as np
import torch
from PIL import Image

from data.image_folder import make_dataset


class AlignedDataset(torch.utils.data.Dataset):
    def initialize(self, opt):
        self.opt = opt
        self.dir_AB = os.path.join(opt.dataroot, opt.phase)
        # sorted() of the (A list, B list) pair, as the reference (:35)
        self.A_paths, self.B_paths = sorted(make_dataset(self.dir_AB))
        assert opt.resize_or_crop == "resize_and_crop"

    def _crop(self, path, h_off, w_off):
        img = np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8)
        fh, fw = self.opt.fineSize_h, self.opt.fineSize_w
        return img[h_off:h_off + fh, w_off:w_off + fw].copy()

    def __getitem__(self, index):
        opt = self.opt
        A_path, B_path = self.A_paths[index], self.B_paths[index]
        w_offset = random.randint(0, max(0, opt.loadSize_w - opt.fineSize_w - 1))
        h_offset = random.randint(0, max(0, opt.loadSize_h - opt.fineSize_h - 1))
        flip = (not opt.no_flip) and random.random() < 0.5
        return {"A_u8": torch.from_numpy(self._crop(A_path, h_offset, w_offset)),
                "B_u8": torch.from_numpy(self._crop(B_path, h_offset, w_offset)),
                "flip": int(flip), "A_paths": A_path, "B_paths": B_path}

    def __len__(self):
        return len(self.A_paths)

    def name(self):
        return "AlignedDataset"
