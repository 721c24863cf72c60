"""History buffer of generated pairs fed to D (DSGAN/util/image_pool.py:5-32).

Same decision rule and the same python-``random`` draws (``uniform(0,1) > 0.5`` then
``randint(0, size-1)``) per image, so a seeded run consumes the RNG exactly like the
reference.  The pool is ONE resident device tensor [pool_size, C, H, W]; a query resolves the
reference's per-image loop on the host (which slot each output image comes from, which slots
take which input image -- the same image may be swapped in and out of one slot twice within a
batch), then runs two batched copies: the output gather (from the input or the pool's
previous contents) and, after it, the scatter of the new images into their slots.
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
            self.store = None          # [pool_size, C, H, W], allocated at the first query

    @property
    def images(self):
        """The stored images, reference order (views of the resident pool)."""
        return [self.store[i:i + 1] for i in range(self.num_imgs)] if self.pool_size > 0 and self.store is not None else []

    def query(self, images, out=None):
        """The reference's query; ``out`` (optional, images' shape): the result is written there (the
        CUDA-graph step's static buffer between its two captured halves)."""
        if self.pool_size == 0:
            if out is not None:
                out.copy_(images)
                return out
            return images
        images = images.detach().contiguous()
        if self.store is not None and (self.store.shape[1:] != images.shape[1:] or self.store.dtype != images.dtype
                                       or self.store.device != images.device):
            if self.num_imgs > 0:
                # the reference's list would mix shapes and its torch.cat (image_pool.py:32) fail
                raise ValueError("ImagePool.query: images of shape %s %s on %s, the pool holds %d of shape %s %s on %s"
                                 % (tuple(images.shape[1:]), images.dtype, images.device, self.num_imgs,
                                    tuple(self.store.shape[1:]), self.store.dtype, self.store.device))
            self.store = None
        if self.store is None:
            self.store = torch.empty((self.pool_size,) + tuple(images.shape[1:]), device=images.device,
                                     dtype=images.dtype)
        # slot -> where its CURRENT contents live: ("pool", slot) = unchanged this query, ("in", j)
        cur = {}
        src_of_out = []
        for i in range(images.shape[0]):
            if self.num_imgs < self.pool_size:
                cur[self.num_imgs] = ("in", i)
                self.num_imgs += 1
                src_of_out.append(("in", i))
            else:
                p = self.rng.uniform(0, 1)
                if p > 0.5:
                    random_id = self.rng.randint(0, self.pool_size - 1)
                    src_of_out.append(cur.get(random_id, ("pool", random_id)))
                    cur[random_id] = ("in", i)
                else:
                    src_of_out.append(("in", i))
        if out is None:
            out = torch.empty_like(images)

        def t(src):
            return images[src[1]] if src[0] == "in" else self.store[src[1]]
        # gather first (it may read slots the scatter below overwrites), then scatter
        HF.copy_multi([(out[i], t(s)) for i, s in enumerate(src_of_out)])
        HF.copy_multi([(self.store[slot], images[j]) for slot, (_, j) in sorted(cur.items())])
        return out
