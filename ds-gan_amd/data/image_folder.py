"""Image listing (DSGAN/data/image_folder.py:13-34).

``make_dataset(dir)`` walks ``dir`` and returns (first half, second half) of the image paths,
as the reference does; unlike the reference the file names inside each directory are sorted,
so the A/B pairing does not depend on the file system's directory order."""
import os

IMG_EXTENSIONS = [".jpg", ".JPG", ".jpeg", ".JPEG", ".png", ".PNG", ".ppm", ".PPM", ".bmp", ".BMP"]


def is_image_file(filename):
    return any(filename.endswith(extension) for extension in IMG_EXTENSIONS)


def make_dataset(dir):
    assert os.path.isdir(dir), "%s is not a valid directory" % dir
    images = []
    for root, _, fnames in sorted(os.walk(dir)):
        for fname in sorted(fnames):
            if is_image_file(fname):
                images.append(os.path.join(root, fname))
    ix = len(images) // 2
    return images[:ix], images[ix:]
