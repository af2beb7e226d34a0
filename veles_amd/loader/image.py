"""Image loaders (PIL).

Reference: veles/loader/image.py:83-806 (ImageLoader: colour space, scale
with aspect keeping, crop, mirror, rotations, background), file_image.py,
fullbatch_image.py, image_mse.py.  MI355X design: images are decoded and
resized once on the host into one uint8 NHWC array that becomes the device-
resident full batch (288 GB of HBM holds ImageNet-scale sets); the per-step
gather + normalisation is the ``fill_minibatch`` kernel of FullBatchLoader.
Augmentation that must vary per epoch (mirror / crop jitter) is done on the
device in ``fill_indices`` with torch flips on the gathered minibatch.
"""
from __future__ import annotations

import numpy

from veles_amd.loader.base import TEST, TRAIN, VALID
from veles_amd.loader.file_loader import (
    FileFilter, label_from_path, read_file_list, scan_files)
from veles_amd.loader.fullbatch import FullBatchLoader, FullBatchLoaderMSE

__all__ = ["decode_image", "FullBatchFileImageLoader",
           "FullBatchAutoLabelFileImageLoader", "FileListImageLoader",
           "FullBatchImageLoaderMSE"]

COLOR_SPACES = {"RGB": 3, "GRAY": 1, "HSV": 3, "YCbCr": 3, "LAB": 3}


def decode_image(path, size=None, color_space="RGB", crop=None,
                 keep_aspect=True, background=0):
    """File -> uint8 HWC array.  ``size`` = (width, height); with
    ``keep_aspect`` the image is scaled to fit and centred on a
    ``background`` canvas; ``crop`` = (left, top, right, bottom) in source
    pixels before scaling."""
    from PIL import Image
    img = Image.open(path)
    mode = {"GRAY": "L", "RGB": "RGB", "HSV": "HSV", "YCbCr": "YCbCr",
            "LAB": "LAB"}[color_space]
    img = img.convert("RGB")
    if crop is not None:
        img = img.crop(tuple(crop))
    if size is not None:
        w, h = size
        if keep_aspect:
            s = min(w / img.width, h / img.height)
            nw, nh = max(1, round(img.width * s)), max(1, round(
                img.height * s))
            img = img.resize((nw, nh), Image.BILINEAR)
            canvas = Image.new("RGB", (w, h), (background,) * 3)
            canvas.paste(img, ((w - nw) // 2, (h - nh) // 2))
            img = canvas
        else:
            img = img.resize((w, h), Image.BILINEAR)
    if mode == "LAB":
        from PIL import ImageCms
        srgb = ImageCms.createProfile("sRGB")
        lab = ImageCms.createProfile("LAB")
        img = ImageCms.profileToProfile(
            img, ImageCms.buildTransformFromOpenProfiles(srgb, lab, "RGB",
                                                         "LAB"))
    elif mode != "RGB":
        img = img.convert(mode)
    a = numpy.asarray(img, dtype=numpy.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    return a


class _ImageMixin(object):
    def _image_kwargs(self, kwargs):
        self.size = tuple(kwargs["size"]) if kwargs.get("size") else None
        self.color_space = kwargs.get("color_space", "RGB")
        if self.color_space not in COLOR_SPACES:
            raise ValueError("color_space must be one of %s" %
                             sorted(COLOR_SPACES))
        self.crop = kwargs.get("crop")
        self.keep_aspect_ratio = kwargs.get("keep_aspect_ratio", True)
        self.background_color = int(kwargs.get("background_color", 0))
        self.mirror = kwargs.get("mirror", False)

    def _decode_all(self, files):
        imgs = [decode_image(f, self.size, self.color_space, self.crop,
                             self.keep_aspect_ratio, self.background_color)
                for f in files]
        if not imgs:
            return numpy.zeros((0, 1, 1, 1), numpy.uint8)
        shape = imgs[0].shape
        for f, im in zip(files, imgs):
            if im.shape != shape:
                raise ValueError("%s has shape %s, expected %s (set size=)" %
                                 (f, im.shape, shape))
        return numpy.stack(imgs)

    def _augment(self):
        """Per-epoch random horizontal mirror of TRAIN minibatches."""
        if not self.mirror or self.minibatch_class != TRAIN:
            return
        import torch
        x = self.minibatch_data.devmem
        n = self.minibatch_size
        flip = torch.rand(n, device=x.device) < 0.5
        if bool(flip.any()):
            x[:n][flip] = torch.flip(x[:n][flip], dims=[2])


class _LabelledFilesLoader(_ImageMixin, FullBatchLoader):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self._image_kwargs(kwargs)
        self.file_filter = FileFilter(
            kwargs.get("mime_types", ("image/",)),
            kwargs.get("filename_types"), kwargs.get("included"),
            kwargs.get("ignored"))
        self.paths = {TEST: kwargs.get("test_paths", ()),
                      VALID: kwargs.get("validation_paths", ()),
                      TRAIN: kwargs.get("train_paths", ())}

    def files_and_labels(self, cls):
        raise NotImplementedError

    def load_data(self):
        datas, labels = [], []
        self.class_lengths = [0, 0, 0]
        for cls in (TEST, VALID, TRAIN):
            fl = self.files_and_labels(cls)
            self.class_lengths[cls] = len(fl)
            if fl:
                datas.append(self._decode_all([f for f, _ in fl]))
                labels.extend(lbl for _, lbl in fl)
        if not datas:
            raise ValueError("%s: no files found" % self)
        data = numpy.concatenate(datas)
        if any(lbl is not None for lbl in labels):
            names = sorted({lbl for lbl in labels if lbl is not None},
                           key=lambda v: (str(type(v)), v))
            self.labels_mapping = {v: i for i, v in enumerate(names)}
            self.reversed_labels_mapping = names
            self.original_labels = numpy.array(
                [self.labels_mapping.get(lbl, -1) for lbl in labels],
                numpy.int32)
        self.original_data.reset(data)
        self._apply_validation_ratio()

    def fill_indices(self, start_offset, count):
        done = super().fill_indices(start_offset, count)
        self._augment()
        return done


class FullBatchFileImageLoader(_LabelledFilesLoader):
    """Directories of images; label = regex group (``label_regexp``) or the
    parent directory name."""
    MAPPING = "full_batch_file_image"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.label_regexp = kwargs.get("label_regexp")

    def files_and_labels(self, cls):
        files = scan_files(self.paths[cls], self.file_filter) \
            if self.paths[cls] else []
        return [(f, label_from_path(f, self.label_regexp)) for f in files]


class FullBatchAutoLabelFileImageLoader(FullBatchFileImageLoader):
    MAPPING = "full_batch_auto_label_file_image"


class FileListImageLoader(_LabelledFilesLoader):
    """Text lists "path label" per class (``test_list`` / ``validation_list``
    / ``train_list``)."""
    MAPPING = "file_list_image"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.lists = {TEST: kwargs.get("test_list"),
                      VALID: kwargs.get("validation_list"),
                      TRAIN: kwargs.get("train_list")}

    def files_and_labels(self, cls):
        lst = self.lists[cls]
        return read_file_list(lst) if lst else []


class FullBatchImageLoaderMSE(_ImageMixin, FullBatchLoaderMSE):
    """Image -> image regression: target = the file of the same base name
    under ``target_paths`` (reference image_mse.py)."""
    MAPPING = "full_batch_image_mse"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self._image_kwargs(kwargs)
        self.file_filter = FileFilter(kwargs.get("mime_types", ("image/",)))
        self.paths = {TEST: kwargs.get("test_paths", ()),
                      VALID: kwargs.get("validation_paths", ()),
                      TRAIN: kwargs.get("train_paths", ())}
        self.target_paths = kwargs["target_paths"]

    def load_data(self):
        import os
        targets = {os.path.splitext(os.path.basename(f))[0]: f
                   for f in scan_files(self.target_paths, self.file_filter)}
        xs, ts = [], []
        self.class_lengths = [0, 0, 0]
        for cls in (TEST, VALID, TRAIN):
            files = scan_files(self.paths[cls], self.file_filter) \
                if self.paths[cls] else []
            pairs = [(f, targets.get(os.path.splitext(
                os.path.basename(f))[0])) for f in files]
            pairs = [(f, t) for f, t in pairs if t is not None]
            self.class_lengths[cls] = len(pairs)
            if pairs:
                xs.append(self._decode_all([f for f, _ in pairs]))
                ts.append(self._decode_all([t for _, t in pairs]))
        self.original_data.reset(numpy.concatenate(xs))
        self.original_targets.reset(numpy.concatenate(ts).astype(
            numpy.float32) / 255.0)
