"""Data loading (DSGAN/data/__init__.py:5-60): ``CreateDataLoader(opt, isTrain)`` ->
``load_data()`` iterable of ``{'A', 'B', 'A_paths', 'B_paths'}`` batches, A/B float32 NCHW in
[-1, 1] already on the GPU (set_input's ``.to(device)`` is then a no-op).

Multi-GPU (one process per GPU under torchrun): ``--batchSize`` keeps the reference's meaning,
the GLOBAL batch that ``nn.DataParallel`` scatters over the GPUs (DSGAN/models/networks.py:74-77,
``Tensor.chunk`` along dim 0).  Every rank walks the same epoch permutation (same seed, same RNG
draws as the 1-GPU loader) and takes its chunk of each global batch (``RankBatchSampler``), so
the sequence of global batches equals the single-process run's.  Each batch dict also carries
``global_batch`` (the size of the global batch it is a chunk of) for the loss weighting of
ragged last batches (Pix2PixModel.set_input).
"""
import collections
import math

import torch
import torch.distributed as dist

from dsgan_hip._lib import call, ptr, stream


def to_images(u8, flip, gray=False):
    """uint8 [N][H][W][3] (host or device) + flip flags -> fp32 [N][3|1][H][W] on the GPU."""
    dev = torch.device("cuda", torch.cuda.current_device())
    u8 = u8.to(dev, non_blocking=True).contiguous()
    fl = torch.as_tensor(flip, dtype=torch.int32).to(dev, non_blocking=True)
    N, H, W, _ = u8.shape
    out = torch.empty((N, 1 if gray else 3, H, W), device=dev, dtype=torch.float32)
    call("dsgan_u8_to_image", ptr(u8), ptr(fl), ptr(out), N, H, W, int(gray), stream())
    return out


def _dist():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


class RankBatchSampler:
    """Global batches of ``sampler`` (batch_size each, the last one ragged), of which this rank
    yields its ``Tensor.chunk`` slice: chunk = ceil(n / world), rank r gets [r*chunk, (r+1)*chunk).
    ``Tensor.chunk`` leaves trailing ranks EMPTY when n <= (world-1)*chunk (e.g. n=4 over 3 GPUs
    gives chunks [2, 2]); a step's collectives need every rank, so such a ragged last batch is
    skipped on every rank, and a batch_size that is itself not viable is refused up front.
    The epoch's index list is drawn on every rank (same RNG consumption as the 1-process loader)
    and rank 0's list is broadcast, so the ranks cannot drift apart.  ``sizes`` queues the global
    size of each yielded chunk, in order."""

    def __init__(self, sampler, batch_size, rank, world):
        self.sampler, self.batch_size, self.rank, self.world = sampler, batch_size, rank, world
        self.sizes = collections.deque()
        if not self.viable(batch_size):
            raise ValueError(
                "--batchSize %d (the global batch) cannot be split over %d ranks: Tensor.chunk would leave "
                "rank(s) without samples (chunk %d); use a batchSize with ceil(B/W)*(W-1) < B, e.g. a multiple of %d"
                % (batch_size, world, math.ceil(batch_size / world), world))

    def viable(self, n):
        """True when every rank gets at least one sample of an n-sample global batch."""
        return n > (self.world - 1) * math.ceil(n / self.world)

    def _chunk(self, buf):
        n = len(buf)
        if not self.viable(n):
            return None
        c = math.ceil(n / self.world)
        return buf[self.rank * c:(self.rank + 1) * c]

    def _epoch_indices(self):
        idx = list(self.sampler)
        if self.world > 1 and dist.is_available() and dist.is_initialized():
            dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() == "nccl" else torch.device("cpu")
            t = torch.tensor(idx, dtype=torch.int64, device=dev)
            dist.broadcast(t, 0)
            idx = t.cpu().tolist()
        return idx

    def __iter__(self):
        self.sizes.clear()
        buf = []
        for idx in self._epoch_indices():
            buf.append(idx)
            if len(buf) == self.batch_size:
                mine = self._chunk(buf)
                if mine is not None:
                    self.sizes.append(len(buf))
                    yield mine
                buf = []
        if buf:
            mine = self._chunk(buf)
            if mine is not None:
                self.sizes.append(len(buf))
                yield mine

    def __len__(self):
        full, tail = divmod(len(self.sampler), self.batch_size)
        return (full if self.viable(self.batch_size) else 0) + (1 if tail and self.viable(tail) else 0)


def CreateDataset(opt):
    if opt.dataset_mode == "aligned":
        from data.aligned_dataset import AlignedDataset
        dataset = AlignedDataset()
    elif opt.dataset_mode == "single":
        from data.single_dataset import SingleDataset
        dataset = SingleDataset()
    else:
        raise ValueError("Dataset [%s] not recognized." % opt.dataset_mode)
    print("dataset [%s] was created" % dataset.name())
    dataset.initialize(opt)
    return dataset


class CustomDatasetDataLoader:
    def name(self):
        return "CustomDatasetDataLoader"

    def initialize(self, opt, isTrain):
        self.opt = opt
        self.dataset = CreateDataset(opt)
        shuffle = (not opt.serial_batches) if isTrain == "train" else False
        rank, world = _dist()
        self.batch_sampler = None
        if world == 1:
            self.dataloader = torch.utils.data.DataLoader(
                self.dataset, batch_size=opt.batchSize, shuffle=shuffle,
                num_workers=int(opt.nThreads), pin_memory=True)
        else:
            # the same sampler (hence the same RNG draws) as the 1-process loader above
            sampler = (torch.utils.data.RandomSampler(self.dataset) if shuffle
                       else torch.utils.data.SequentialSampler(self.dataset))
            self.batch_sampler = RankBatchSampler(sampler, opt.batchSize, rank, world)
            self.dataloader = torch.utils.data.DataLoader(
                self.dataset, batch_sampler=self.batch_sampler, num_workers=int(opt.nThreads),
                pin_memory=True)

    def load_data(self):
        return self

    def __len__(self):
        return min(len(self.dataset), self.opt.max_dataset_size)

    def __iter__(self):
        opt = self.opt
        AtoB = opt.which_direction == "AtoB"
        in_nc, out_nc = (opt.input_nc, opt.output_nc) if AtoB else (opt.output_nc, opt.input_nc)
        for i, data in enumerate(self.dataloader):
            if i * opt.batchSize >= opt.max_dataset_size:
                break
            gb = self.batch_sampler.sizes.popleft() if self.batch_sampler is not None else len(data["A_paths"])
            if "B_u8" not in data:     # single dataset (--model test): A only
                yield {"A": to_images(data["A_u8"], data["flip"], in_nc == 1), "A_paths": data["A_paths"],
                       "global_batch": gb}
                continue
            yield {"A": to_images(data["A_u8"], data["flip"], in_nc == 1),
                   "B": to_images(data["B_u8"], data["flip"], out_nc == 1),
                   "A_paths": data["A_paths"], "B_paths": data["B_paths"], "global_batch": gb}


def CreateDataLoader(opt, isTrain="train"):
    data_loader = CustomDatasetDataLoader()
    print(data_loader.name())
    data_loader.initialize(opt, isTrain)
    return data_loader
