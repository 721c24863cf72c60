"""History buffer of generated pairs fed to D (DSGAN/util/image_pool.py:5-32).

Same decision rule and the same python-``random`` draws (``uniform(0,1) > 0.5`` then
``randint(0, size-1)``) per image, so a seeded run consumes the RNG exactly like the
reference.  Images stay on the device; copies go through the HIP strided-copy kernel.
"""
import random

import torch

from dsgan_hip import functional as HF


class ImagePool:
    def __init__(self, pool_size, rng=None):
        self.pool_size = pool_size
        self.rng = rng if rng is not None else random
        if self.pool_size > 0:
            self.num_imgs = 0
            self.images = []

    @staticmethod
    def _clone(img):
        out = torch.empty_like(img)
        HF.copy_into(out, img)
        return out

    def query(self, images):
        if self.pool_size == 0:
            return images
        images = images.detach()
        picks = []
        for i in range(images.shape[0]):
            image = images[i:i + 1]
            if self.num_imgs < self.pool_size:
                self.num_imgs += 1
                stored = self._clone(image)
                self.images.append(stored)
                picks.append(stored)
            else:
                p = self.rng.uniform(0, 1)
                if p > 0.5:
                    random_id = self.rng.randint(0, self.pool_size - 1)
                    tmp = self.images[random_id]
                    self.images[random_id] = self._clone(image)
                    picks.append(tmp)
                else:
                    picks.append(image)
        out = torch.empty_like(images)
        for i, t in enumerate(picks):
            HF.copy_into(out[i:i + 1], t)
        return out
