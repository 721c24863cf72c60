"""Data loading (DSGAN/data/__init__.py:5-60): ``CreateDataLoader(opt, isTrain)`` ->
``load_data()`` iterable of ``{'A', 'B', 'A_paths', 'B_paths'}`` batches, A/B float32 NCHW in
[-1, 1] already on the GPU (set_input's ``.to(device)`` is then a no-op)."""
import torch

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


def CreateDataset(opt):
    if opt.dataset_mode != "aligned":
        raise ValueError("Dataset [%s] not recognized." % opt.dataset_mode)
    from data.aligned_dataset import AlignedDataset
    dataset = AlignedDataset()
    print("dataset [%s] was created" % dataset.name())
    dataset.initialize(opt)
    return dataset


class CustomDatasetDataLoader:
    def name(self):
        return "CustomDatasetDataLoader"

    def initialize(self, opt, isTrain):
        self.opt = opt
        self.dataset = CreateDataset(opt)
        self.dataloader = torch.utils.data.DataLoader(
            self.dataset, batch_size=opt.batchSize,
            shuffle=(not opt.serial_batches) if isTrain == "train" else False,
            num_workers=int(opt.nThreads), pin_memory=True)

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
            yield {"A": to_images(data["A_u8"], data["flip"], in_nc == 1),
                   "B": to_images(data["B_u8"], data["flip"], out_nc == 1),
                   "A_paths": data["A_paths"], "B_paths": data["B_paths"]}


def CreateDataLoader(opt, isTrain="train"):
    data_loader = CustomDatasetDataLoader()
    print(data_loader.name())
    data_loader.initialize(opt, isTrain)
    return data_loader
