"""Single-image dataset for ``--model test`` (DSGAN/data/single_dataset.py:7-41).

The reference's SingleDataset cannot run as written: ``make_dataset`` returns the (A half,
B half) pair of one directory walk (DSGAN/data/image_folder.py:24-34), so ``A_paths[index]`` is
a whole list, and ``get_transform`` reads ``opt.loadSize`` / ``opt.fineSize``, which the option
table does not define (only ``*_w`` / ``*_h``, DSGAN/options/base_options.py:22-25).  The build
serves what the class evidently intends -- the A (TIR) half of ``dataroot``, sorted -- through
the same uint8 upload + ``dsgan_u8_to_image`` kernel as the aligned dataset, cropped to
``fineSize_h x fineSize_w`` at python-``random`` offsets and never flipped (``isTrain`` is False
at test time, DSGAN/data/base_dataset.py:33); RGB -> gray when ``input_nc == 1`` (:25-27).
"""
import os
import random

import numpy as np
import torch
from PIL import Image

from data.image_folder import make_dataset


class SingleDataset(torch.utils.data.Dataset):
    def initialize(self, opt):
        self.opt = opt
        self.root = opt.dataroot
        self.dir_A = os.path.join(opt.dataroot)
        self.A_paths = sorted(make_dataset(self.dir_A)[0])

    def __getitem__(self, index):
        opt = self.opt
        A_path = self.A_paths[index]
        img = np.asarray(Image.open(A_path).convert("RGB"), dtype=np.uint8)
        fh, fw = opt.fineSize_h, opt.fineSize_w
        w_offset = random.randint(0, max(0, img.shape[1] - fw))
        h_offset = random.randint(0, max(0, img.shape[0] - fh))
        crop = img[h_offset:h_offset + fh, w_offset:w_offset + fw].copy()
        if crop.shape[:2] != (fh, fw):
            raise ValueError("SingleDataset: %s is %dx%d, smaller than fineSize %dx%d"
                             % (A_path, img.shape[0], img.shape[1], fh, fw))
        return {"A_u8": torch.from_numpy(crop), "flip": 0, "A_paths": A_path}

    def __len__(self):
        return len(self.A_paths)

    def name(self):
        return "SingleImageDataset"
