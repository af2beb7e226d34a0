"""Image loaders: full-batch (every canvas resident in HBM) and streaming
(decoded on demand by host workers, prefetched, copied asynchronously).

Reference: veles/loader/image.py:106-806 (ImageLoader: colour space, scale
with aspect keeping onto a background, crop / crop_number / smart_crop,
mirror, rotations, Sobel channel, background image, samples_inflation),
file_image.py:53-183 (FileImageLoader, FileListImageLoader,
AutoLabelFileImageLoader), fullbatch_image.py (the FullBatch* variants,
which materialise every distorted copy at load time), image_mse.py.

MI355X design:

* a *canvas* is one decoded, scaled image (uint8 HWC, ``size`` = (width,
  height) with the aspect kept on the background); canvases are the only
  pixels the host produces;
* every served sample is (canvas, distortion slot): ``samples_inflation``
  slots per canvas (loader/augment.py), so one canvas yields its mirrored /
  rotated / re-cropped variants without being stored more than once;
* the crop, mirror, rotation, background fill, Sobel channel and the
  normaliser's per-feature affine map run on the device in ONE kernel per
  minibatch (``ops.image_batch`` / hvk_image_batch) from parameters the
  loader's PRNG draws on the host: reproducible from ``-r`` and with no
  device -> host synchronisation;
* full-batch loaders keep all canvases in HBM (288 GB per GPU) and gather
  from them; the streaming ``ImageLoader`` decodes a minibatch's canvases
  in a host thread pool into pinned memory, copies them on a side stream
  and makes the compute stream wait on an event, while the NEXT minibatch
  (predicted from the serving state machine) is already being decoded:
  loader / compute overlap;
* label bookkeeping and the label-stratified validation split come from
  loader/labels.py.
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import threading

import numpy

from veles_amd.error import BadFormatError
from veles_amd.loader.augment import Augmentation
from veles_amd.loader.base import Loader, TEST, TRAIN, VALID
from veles_amd.loader.file_loader import (
    FileFilter, label_from_path, read_file_list, scan_files)
from veles_amd.loader.fullbatch import FullBatchLoader, FullBatchLoaderMSE

__all__ = ["decode_image", "ImageLoader", "FileImageLoader",
           "AutoLabelFileImageLoader", "FileListImageLoader",
           "FullBatchFileImageLoader", "FullBatchAutoLabelFileImageLoader",
           "FullBatchFileListImageLoader", "FullBatchImageLoaderMSE"]

COLOR_SPACES = {"RGB": 3, "GRAY": 1, "HSV": 3, "YCbCr": 3, "LAB": 3}


def _bg_tuple(background, channels):
    if background is None:
        return (0,) * channels
    if isinstance(background, (int, numpy.integer)):
        return (int(background),) * channels
    bg = tuple(int(v) for v in background)
    if len(bg) == 1:
        return bg * channels
    if len(bg) != channels:
        raise ValueError("background_color %r does not match %d channels" %
                         (background, channels))
    return bg


def decode_image(path, size=None, color_space="RGB", crop=None,
                 keep_aspect=True, background=0, background_image=None):
    """File -> uint8 HWC canvas.  ``size`` = (width, height); with
    ``keep_aspect`` the image is scaled to fit and centred on the background
    (``background_image`` [H][W][C] uint8, else the ``background`` colour);
    ``crop`` = (left, top, right, bottom) in source pixels before scaling."""
    from PIL import Image
    img = Image.open(path)
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
            if background_image is not None:
                canvas = Image.fromarray(numpy.asarray(
                    background_image, numpy.uint8)[:, :, :3]).convert("RGB")
            else:
                canvas = Image.new("RGB", (w, h), _bg_tuple(background, 3))
            canvas.paste(img, ((w - nw) // 2, (h - nh) // 2))
            img = canvas
        else:
            img = img.resize((w, h), Image.BILINEAR)
    if color_space == "LAB":
        from PIL import ImageCms
        srgb = ImageCms.createProfile("sRGB")
        lab = ImageCms.createProfile("LAB")
        img = ImageCms.profileToProfile(
            img, ImageCms.buildTransformFromOpenProfiles(srgb, lab, "RGB",
                                                         "LAB"))
    elif color_space != "RGB":
        img = img.convert({"GRAY": "L", "HSV": "HSV",
                           "YCbCr": "YCbCr"}[color_space])
    a = numpy.asarray(img, dtype=numpy.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    return a


class _ImageMixin(object):
    """Canvas / augmentation / normalisation plumbing shared by the
    full-batch and the streaming image loaders."""

    def _image_kwargs(self, kwargs):
        self.size = tuple(kwargs["size"]) if kwargs.get("size") else None
        self.color_space = kwargs.get("color_space", "RGB")
        if self.color_space not in COLOR_SPACES:
            raise ValueError("color_space must be one of %s" %
                             sorted(COLOR_SPACES))
        self.source_crop = kwargs.get("source_crop")
        self.keep_aspect_ratio = kwargs.get(
            "keep_aspect_ratio", kwargs.get("scale_maintain_aspect_ratio",
                                            True))
        self.background_color = kwargs.get("background_color", 0)
        bgi = kwargs.get("background_image")
        if isinstance(bgi, str):
            from PIL import Image
            bgi = numpy.asarray(Image.open(bgi).convert("RGB"), numpy.uint8)
        self.background_image = bgi
        self.augment = Augmentation(
            crop=kwargs.get("crop"), crop_number=kwargs.get("crop_number", 1),
            mirror=kwargs.get("mirror", False),
            rotations=kwargs.get("rotations", (0.0,)),
            smart_crop=kwargs.get("smart_crop", True),
            add_sobel=kwargs.get("add_sobel", False))

    @property
    def channels_number(self):
        return COLOR_SPACES[self.color_space]

    def decode(self, path):
        return decode_image(path, self.size, self.color_space,
                            self.source_crop, self.keep_aspect_ratio,
                            self.background_color,
                            self.background_image
                            if self.size is not None else None)

    def get_image_bbox(self, key, size):
        """(ymin, ymax, xmin, xmax) of the object in a canvas (smart crop);
        the whole canvas unless overridden."""
        return 0, size[0], 0, size[1]

    @property
    def canvas_shape(self):
        return tuple(self.canvas_shape_)

    @property
    def served_shape(self):
        H, W, C = self.canvas_shape
        h, w = self.augment.output_hw((H, W))
        return h, w, self.augment.channels(C)

    def _bg_for_output(self):
        """(bg uint8 [Ho][Wo][C] or None, bgcolor float32 [C]) used where a
        rotation reaches outside the crop."""
        h, w, _ = self.served_shape
        C = self.canvas_shape[2]
        bg = None
        if self.background_image is not None:
            b = numpy.asarray(self.background_image, numpy.uint8)
            if b.ndim == 2:
                b = b[:, :, None]
            bg = numpy.ascontiguousarray(b[:h, :w, :C])
            if bg.shape != (h, w, C):
                raise BadFormatError("background_image %s is smaller than a "
                                     "served sample %s" % (b.shape, (h, w)))
        color = numpy.asarray(_bg_tuple(self.background_color, C),
                              numpy.float32)
        return bg, color

    def _affine_served(self):
        """The normaliser's (mean, rdisp) broadcast over a served sample,
        float32 [Ho*Wo*Co] each, or (None, None)."""
        if self.normalizer is None or self.normalization_type == "none":
            return None, None
        aff = self.normalizer.affine()
        if aff is None:
            raise BadFormatError(
                "%s: image loaders apply the normaliser on the device and "
                "need an affine one (mean_disp, linear, range_linear, "
                "pointwise, external_mean, internal_mean), not %s" %
                (self, self.normalization_type))
        feat = int(numpy.prod(self.served_shape))
        return tuple(numpy.broadcast_to(
            numpy.asarray(a, numpy.float32), (feat,)).copy() for a in aff)

    def _served_center(self, canvases):
        """Centre-cropped (+ Sobel) float32 samples of host canvases, the
        exact device transform on the CPU: what the normaliser analyses."""
        import torch
        from veles_amd import ops
        src = torch.from_numpy(numpy.ascontiguousarray(canvases))
        n = len(canvases)
        p = torch.from_numpy(self.augment.params(
            self.canvas_shape[:2], numpy.zeros(n, numpy.int64), None,
            center=True))
        h, w, _ = self.served_shape
        bg, color = self._bg_for_output()
        return ops.image_batch_ref(
            src, torch.arange(n, dtype=torch.int32), p, h, w,
            sobel=self.augment.add_sobel,
            bg=None if bg is None else torch.from_numpy(bg),
            bgcolor=torch.from_numpy(color)).numpy()

    def _device_extras(self, tdev):
        import torch
        mean, rdisp = self._affine_served()
        bg, color = self._bg_for_output()
        to = (lambda a: None if a is None else
              torch.from_numpy(numpy.ascontiguousarray(a)).to(tdev))
        self._dev_img_ = {"mean": to(mean), "rdisp": to(rdisp),
                          "bg": to(bg), "bgcolor": to(color)}

    def _image_batch(self, canvases, idx, params, out):
        from veles_amd import ops
        e = self._dev_img_
        ops.image_batch(canvases, idx, params, out,
                        sobel=self.augment.add_sobel, mean=e["mean"],
                        rdisp=e["rdisp"], bg=e["bg"], bgcolor=e["bgcolor"])

    def _split_sample(self, sample_idx):
        """(canvas-level position, distortion slot) of inflated indices."""
        infl = self.augment.samples_inflation
        a = numpy.asarray(sample_idx, numpy.int64)
        return a // infl, a % infl

    def _rank_params(self, start_offset, count, slot_bbox):
        """Augmentation parameters of this rank's ``count`` samples from
        ``start_offset``: drawn for the whole GLOBAL minibatch and sliced,
        so every rank draws the same sequence from the workflow PRNG and N
        ranks augment exactly as one process over the global minibatch.
        ``slot_bbox(sample) -> (distortion slot, bbox)``."""
        gsize = int(getattr(self, "global_minibatch_size", 0) or 0)
        b = 0
        if gsize > count:
            b, _ = self.shard_bounds(gsize)
        else:
            gsize = count
        g0 = start_offset - b
        samples = self.shuffled_indices.mem[g0:g0 + gsize]
        sb = [slot_bbox(int(v)) for v in samples]
        H, W = self.canvas_shape[:2]
        p = self.augment.params((H, W), [x[0] for x in sb], self.prng,
                                [x[1] for x in sb])
        return p[b:b + count]


# ------------------------------------------------------------- full batch
class _FullBatchImages(_ImageMixin, FullBatchLoader):
    """All canvases resident on the device; samples are (canvas, slot)
    pairs gathered, distorted and normalised by one kernel per minibatch."""
    hide_from_registry = True
    BUILDS_LABELS_MAPPING = True

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self._image_kwargs(kwargs)

    def init_unpickled(self):
        super().init_unpickled()
        self._dev_img_ = None
        self.canvas_order_ = None

    @property
    def sample_shape(self):
        return self.served_shape

    def set_canvases(self, data, labels, class_counts):
        """Install decoded canvases (uint8 [n][H][W][C], TEST | VALID |
        TRAIN) and their raw labels; splits the validation set over the
        canvases, then inflates every class by the distortion slots."""
        self.canvas_shape_ = tuple(data.shape[1:])
        self.class_lengths = list(class_counts)
        if labels is not None and any(lbl is not None for lbl in labels):
            if any(lbl is None for lbl in labels):
                raise BadFormatError("some images have labels, others not")
            self.raw_labels_ = list(labels)
            names = sorted(set(labels), key=lambda v: (str(type(v)), v)) \
                if not self.labels_mapping else None
            if names is not None:
                # provisional: setup_label_stats rebuilds it from TRAIN
                self.labels_mapping = {v: i for i, v in enumerate(names)}
                self.reversed_labels_mapping = names
        else:
            self.raw_labels_ = None
        self.original_data.reset(data)
        lo = self.class_lengths[TEST]
        self.split_validation(self.raw_labels_[lo:]
                              if self.raw_labels_ is not None else None)
        self.canvas_order_ = self.initial_order()
        infl = self.augment.samples_inflation
        self.initial_order_ = (self.canvas_order_.astype(numpy.int64)[:, None]
                               * infl + numpy.arange(infl)).reshape(-1) \
            .astype(self.INDEX_DTYPE)
        self.class_lengths = [n * infl for n in self.class_lengths]

    @property
    def has_labels(self):
        return getattr(self, "raw_labels_", None) is not None

    @has_labels.setter
    def has_labels(self, value):
        pass

    def class_labels(self):
        order = self.initial_order()
        infl = self.augment.samples_inflation
        out, start = [], 0
        for n in self.class_lengths:
            imgs = order[start:start + n:infl] // infl
            out.append([self.raw_labels_[i] for i in imgs])
            start += n
        return out

    def setup_label_stats(self):
        super().setup_label_stats()
        if self.has_labels:
            self.original_labels = numpy.array(
                [self.labels_mapping[v] for v in self.raw_labels_],
                numpy.int32)

    def analyze_dataset(self):
        if self.normalizer is None or self.normalization_type == "none":
            self._affine = None
            return
        infl = self.augment.samples_inflation
        start = sum(self.class_lengths[:TRAIN])
        rows = numpy.unique(self.initial_order()[
            start:start + self.class_lengths[TRAIN]] // infl)
        data = self.original_data.mem
        for i in range(0, len(rows), 256):
            self.normalizer.analyze(self._served_center(data[rows[i:i + 256]]))
        self._affine = None

    def apply_derived_normalization(self):
        self._affine = None

    def create_minibatch_data(self):
        import torch
        n = self.local_minibatch_size
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        self.minibatch_data.devmem = torch.zeros(
            (n,) + self.served_shape, dtype=self._torch_dtype_for_minibatch(),
            device=tdev)
        for arr in (self.minibatch_labels, self.minibatch_indices):
            if arr.mem is not None:
                arr.initialize(dev)

    def on_initialized(self, **kwargs):
        import torch
        super().on_initialized(**kwargs)
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        self._device_extras(tdev)

    def fill_indices(self, start_offset, count):
        import torch
        if self._dev_img_ is None:
            self.on_initialized()
        n = self.local_minibatch_size
        idx = numpy.full(n, -1, numpy.int32)
        idx[:count] = self.shuffled_indices.mem[start_offset:
                                                start_offset + count]
        img, slot = self._split_sample(idx[:count])
        canv = numpy.full(n, -1, numpy.int32)
        canv[:count] = img
        params = numpy.zeros((n, 6), numpy.float32)
        params[:, 2] = 1.0
        if count:
            H, W = self.canvas_shape[:2]

            def slot_bbox(sample):
                im, sl = self._split_sample([sample])
                return int(sl[0]), self.get_image_bbox(int(im[0]), (H, W))
            params[:count] = self._rank_params(start_offset, count,
                                               slot_bbox)
        tdev = self.minibatch_data.devmem.device
        to = (lambda a: torch.from_numpy(a).to(tdev, non_blocking=True)
              if tdev.type != "cpu" else torch.from_numpy(a))
        self._image_batch(self.original_data.devmem, to(canv), to(params),
                          self.minibatch_data.devmem)
        if self.has_labels and self.minibatch_labels.devmem is not None:
            lab = numpy.full(n, -1, numpy.int32)
            lab[:count] = numpy.asarray(self.original_labels)[img]
            self.minibatch_labels.devmem.copy_(to(lab))
        if self.minibatch_indices.devmem is not None:
            self.minibatch_indices.devmem.copy_(to(idx))
        return True


class _LabelledFilesLoader(_FullBatchImages):
    hide_from_registry = True

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.file_filter = FileFilter(
            kwargs.get("mime_types", ("image/",)),
            kwargs.get("filename_types"), kwargs.get("included"),
            kwargs.get("ignored"))
        self.paths = {TEST: kwargs.get("test_paths", ()),
                      VALID: kwargs.get("validation_paths", ()),
                      TRAIN: kwargs.get("train_paths", ())}
        self.decode_workers = int(kwargs.get("decode_workers", min(
            8, os.cpu_count() or 1)))

    def files_and_labels(self, cls):
        raise NotImplementedError

    def load_data(self):
        datas, labels, counts = [], [], [0, 0, 0]
        for cls in (TEST, VALID, TRAIN):
            fl = self.files_and_labels(cls)
            counts[cls] = len(fl)
            if fl:
                with cf.ThreadPoolExecutor(self.decode_workers) as ex:
                    imgs = list(ex.map(self.decode, [f for f, _ in fl]))
                shape = imgs[0].shape
                for (f, _), im in zip(fl, imgs):
                    if im.shape != shape:
                        raise BadFormatError(
                            "%s has shape %s, expected %s (set size=)" %
                            (f, im.shape, shape))
                datas.append(numpy.stack(imgs))
                labels.extend(lbl for _, lbl in fl)
        if not datas:
            raise ValueError("%s: no files found" % self)
        self.set_canvases(numpy.concatenate(datas), labels, counts)


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


class FullBatchFileListImageLoader(_LabelledFilesLoader):
    """Text lists "path label" per class (``test_list`` / ``validation_list``
    / ``train_list``)."""
    MAPPING = "full_batch_file_list_image"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.lists = {TEST: kwargs.get("test_list"),
                      VALID: kwargs.get("validation_list"),
                      TRAIN: kwargs.get("train_list")}

    def files_and_labels(self, cls):
        lst = self.lists[cls]
        return read_file_list(lst) if lst else []


# -------------------------------------------------------------- streaming
class _Staging(object):
    """Two pinned host canvas buffers + their device twins, and the events
    that say when a buffer's host -> device copy has finished."""

    def __init__(self, n, shape, tdev):
        import torch
        gpu = tdev.type == "cuda"
        self.host = [torch.empty((n,) + shape, dtype=torch.uint8,
                                 pin_memory=gpu) for _ in range(2)]
        self.dev = [torch.empty((n,) + shape, dtype=torch.uint8, device=tdev)
                    if gpu else self.host[i] for i in range(2)]
        self.copied = [None, None]
        # recorded on the compute stream after the device twin was last read:
        # the next copy into that twin waits for it on the copy stream
        self.consumed = [None, None]
        self.stream = torch.cuda.Stream(tdev) if gpu else None
        self.gpu = gpu

    def wait_free(self, slot):
        ev = self.copied[slot]
        if ev is not None:
            ev.synchronize()


class ImageLoader(_ImageMixin, Loader):
    """Streaming image loader (reference veles/loader/image.py:106-806).
    Subclasses name the keys of each class and how to read a key's label;
    canvases are decoded when a minibatch needs them, by ``decode_workers``
    host threads, and the next minibatch is prefetched while the current
    one trains (``prefetch``)."""
    hide_from_registry = True
    BUILDS_LABELS_MAPPING = True

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self._image_kwargs(kwargs)
        self.validation_ratio = kwargs.get("validation_ratio")
        self.decode_workers = int(kwargs.get("decode_workers", min(
            8, os.cpu_count() or 1)))
        self.prefetch = bool(kwargs.get("prefetch", True))
        self.class_keys = [[], [], []]
        self.canvas_shape_ = None

    def init_unpickled(self):
        super().init_unpickled()
        self._pool_ = None
        # prefetch jobs run here, not on _pool_: a job that waits on the
        # decode pool from inside it would hold one of its workers (and
        # deadlock with decode_workers=1)
        self._prefetch_pool_ = None
        self._stage_ = None
        self._pending_ = {}
        self._slot_ = 0
        self._dev_img_ = None
        self._lock_ = threading.Lock()
        self.prefetch_hits = 0
        self.prefetch_misses = 0

    # -- subclass API --------------------------------------------------------
    def get_keys(self, cls):
        raise NotImplementedError

    def get_image_label(self, key):
        return None

    def get_image_data(self, key):
        return self.decode(key)

    # -- loading -------------------------------------------------------------
    @property
    def sample_shape(self):
        return self.served_shape

    def load_data(self):
        for cls in (TEST, VALID, TRAIN):
            self.class_keys[cls] = sorted(set(self.get_keys(cls)))
        keys = [k for ks in self.class_keys for k in ks]
        if not keys:
            raise ValueError("%s: no images found" % self)
        labels = [self.get_image_label(k) for k in keys]
        if any(lbl is not None for lbl in labels) and \
                any(lbl is None for lbl in labels):
            raise BadFormatError("some images have labels, others not")
        self._key_labels_ = dict(zip(keys, labels)) \
            if labels[0] is not None else None
        self.has_labels = self._key_labels_ is not None
        self.canvas_shape_ = tuple(self.get_image_data(keys[0]).shape)
        ratio = self.validation_ratio
        if ratio is not None:
            pool = self.class_keys[VALID] + self.class_keys[TRAIN]
            if ratio <= 0:
                self.class_keys[VALID], self.class_keys[TRAIN] = [], pool
            else:
                from veles_amd.loader.labels import (random_split,
                                                     stratified_split)
                if self.has_labels:
                    v, t = stratified_split(
                        [self._key_labels_[k] for k in pool], ratio,
                        self.prng)
                else:
                    v, t = random_split(len(pool), ratio, self.prng)
                self.class_keys[VALID] = [pool[i] for i in v]
                self.class_keys[TRAIN] = [pool[i] for i in t]
        infl = self.augment.samples_inflation
        self.class_lengths = [len(k) * infl for k in self.class_keys]

    def class_labels(self):
        return [[self._key_labels_[k] for k in ks] for ks in self.class_keys]

    def _key_of(self, sample):
        """(key, slot) of an (inflated) global sample index."""
        infl = self.augment.samples_inflation
        cls, rem = self.class_index_by_sample_index(int(sample))
        pos = self.class_lengths[cls] - rem
        return self.class_keys[cls][pos // infl], pos % infl

    def analyze_dataset(self):
        if self.normalizer is None or self.normalization_type == "none":
            return
        keys = self.class_keys[TRAIN]
        with cf.ThreadPoolExecutor(self.decode_workers) as ex:
            for i in range(0, len(keys), 256):
                canv = list(ex.map(self.get_image_data, keys[i:i + 256]))
                self.normalizer.analyze(self._served_center(numpy.stack(
                    canv)))

    def create_minibatch_data(self):
        import torch
        n = self.local_minibatch_size
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        gpu = dev is not None and getattr(dev, "is_gpu", False)
        self.minibatch_data.devmem = torch.zeros(
            (n,) + self.served_shape,
            dtype=dev.compute_dtype if gpu else torch.float32, device=tdev)
        for arr in (self.minibatch_labels, self.minibatch_indices):
            if arr.mem is not None:
                arr.initialize(dev)

    def on_initialized(self, **kwargs):
        import torch
        dev = self.device
        tdev = dev.torch_device if dev is not None else torch.device("cpu")
        self._device_extras(tdev)
        self._stage_ = _Staging(self.local_minibatch_size, self.canvas_shape,
                                tdev)
        if self._pool_ is None:
            self._pool_ = cf.ThreadPoolExecutor(
                self.decode_workers, thread_name_prefix="image-decode")
        if self._prefetch_pool_ is None:
            self._prefetch_pool_ = cf.ThreadPoolExecutor(
                1, thread_name_prefix="image-prefetch")

    def stop(self):
        if self._prefetch_pool_ is not None:
            self._prefetch_pool_.shutdown(wait=True)
            self._prefetch_pool_ = None
        if self._pool_ is not None:
            self._pool_.shutdown(wait=True)
            self._pool_ = None
        super().stop()

    # -- serving -------------------------------------------------------------
    def _decode_into(self, slot, samples):
        """Decode the canvases of ``samples`` into pinned buffer ``slot``
        (waits until that buffer's previous copy to the device is done)."""
        st = self._stage_
        st.wait_free(slot)
        host = st.host[slot].numpy()
        keys = [self._key_of(s)[0] for s in samples]
        for i, c in enumerate(self._pool_.map(self.get_image_data, keys)):
            if c.shape != self.canvas_shape:
                raise BadFormatError("%s: canvas %s, expected %s (set size=)"
                                     % (keys[i], c.shape, self.canvas_shape))
            host[i] = c
        return slot

    def _predict_next(self):
        """Sample indices of the minibatch this rank will serve next, or
        None when it cannot be known now (end of pass: reshuffle; failed
        minibatches pending)."""
        if self.failed_minibatches:
            return None
        off = self.global_offset
        if off >= self.effective_total_samples:
            return None
        _, rem = self.class_index_by_sample_index(off)
        size = min(rem, self.max_minibatch_size)
        b, e = self.shard_bounds(size)
        return tuple(int(v) for v in
                     self.shuffled_indices.mem[off + b:off + e])

    def fill_indices(self, start_offset, count):
        import torch
        if self._stage_ is None or self._pool_ is None:
            self.on_initialized()
        st = self._stage_
        samples = tuple(int(v) for v in
                        self.shuffled_indices.mem[start_offset:
                                                  start_offset + count])
        fut = self._pending_.pop(samples, None)
        if fut is not None:
            slot = fut.result()
            self.prefetch_hits += 1
        else:
            for f in self._pending_.values():   # a stale prediction
                f.result()
            self._pending_.clear()
            self.prefetch_misses += 1
            slot = self._slot_
            self._decode_into(slot, samples)
        n = self.local_minibatch_size
        tdev = self.minibatch_data.devmem.device
        cur = torch.cuda.current_stream(tdev) if st.gpu else None
        if st.gpu:
            if st.consumed[slot] is not None:
                # the compute stream may still be reading this twin (the host
                # can run two minibatches ahead of the GPU)
                st.stream.wait_event(st.consumed[slot])
            with torch.cuda.stream(st.stream):
                st.dev[slot][:count].copy_(st.host[slot][:count],
                                           non_blocking=True)
                ev = torch.cuda.Event()
                ev.record(st.stream)
            st.copied[slot] = ev
            cur.wait_event(ev)
        canv = numpy.full(n, -1, numpy.int32)
        canv[:count] = numpy.arange(count)
        params = numpy.zeros((n, 6), numpy.float32)
        params[:, 2] = 1.0
        if count:
            H, W = self.canvas_shape[:2]

            def slot_bbox(sample):
                key, sl = self._key_of(sample)
                return sl, self.get_image_bbox(key, (H, W))
            params[:count] = self._rank_params(start_offset, count,
                                               slot_bbox)
        to = (lambda a: torch.from_numpy(a).pin_memory().to(
            tdev, non_blocking=True) if st.gpu else torch.from_numpy(a))
        self._image_batch(st.dev[slot], to(canv), to(params),
                          self.minibatch_data.devmem)
        if st.gpu:
            done = torch.cuda.Event()
            done.record(cur)
            st.consumed[slot] = done
        if self.has_labels and self.minibatch_labels.devmem is not None:
            lab = numpy.full(n, -1, numpy.int32)
            lab[:count] = [self.labels_mapping[self._key_labels_[
                self._key_of(s)[0]]] for s in samples]
            self.minibatch_labels.devmem.copy_(to(lab))
        if self.minibatch_indices.devmem is not None:
            idx = numpy.full(n, -1, numpy.int32)
            idx[:count] = samples
            self.minibatch_indices.devmem.copy_(to(idx))
        # the next minibatch decodes into the other buffer meanwhile
        self._slot_ = slot ^ 1
        if self.prefetch:
            nxt = self._predict_next()
            if nxt:
                self._pending_[nxt] = self._prefetch_pool_.submit(
                    self._decode_into, self._slot_, nxt)
        return True


class FileImageLoader(ImageLoader):
    """Streaming loader over directories (``train_paths`` ...); label = regex
    group (``label_regexp``) of the file name or its directory name
    (reference file_image.py:150-183)."""
    MAPPING = "file_image"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.file_filter = FileFilter(
            kwargs.get("mime_types", ("image/",)),
            kwargs.get("filename_types"), kwargs.get("included"),
            kwargs.get("ignored"))
        self.paths = {TEST: kwargs.get("test_paths", ()),
                      VALID: kwargs.get("validation_paths", ()),
                      TRAIN: kwargs.get("train_paths", ())}
        self.label_regexp = kwargs.get("label_regexp")
        self.with_labels = kwargs.get("labels", True)

    def get_keys(self, cls):
        return scan_files(self.paths[cls], self.file_filter) \
            if self.paths[cls] else []

    def get_image_label(self, key):
        return label_from_path(key, self.label_regexp) \
            if self.with_labels else None


class AutoLabelFileImageLoader(FileImageLoader):
    MAPPING = "auto_label_file_image"


class FileListImageLoader(ImageLoader):
    """Streaming loader over "path [label]" lists (``train_list`` ...;
    reference file_image.py:130-148)."""
    MAPPING = "file_list_image"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.lists = {TEST: kwargs.get("test_list"),
                      VALID: kwargs.get("validation_list"),
                      TRAIN: kwargs.get("train_list")}
        self._labels = {}

    def get_keys(self, cls):
        lst = self.lists[cls]
        pairs = read_file_list(lst) if lst else []
        self._labels.update(pairs)
        return [p for p, _ in pairs]

    def get_image_label(self, key):
        return self._labels.get(key)


class FullBatchImageLoaderMSE(_ImageMixin, FullBatchLoaderMSE):
    """Image -> image regression: target = the file of the same base name
    under ``target_paths`` (reference image_mse.py); no geometric
    augmentation (input and target must stay aligned)."""
    MAPPING = "full_batch_image_mse"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self._image_kwargs(kwargs)
        if not self.augment.is_identity:
            raise ValueError("full_batch_image_mse does not augment")
        self.file_filter = FileFilter(kwargs.get("mime_types", ("image/",)))
        self.paths = {TEST: kwargs.get("test_paths", ()),
                      VALID: kwargs.get("validation_paths", ()),
                      TRAIN: kwargs.get("train_paths", ())}
        self.target_paths = kwargs["target_paths"]

    def load_data(self):
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
                xs.append(numpy.stack([self.decode(f) for f, _ in pairs]))
                ts.append(numpy.stack([self.decode(t) for _, t in pairs]))
        self.original_data.reset(numpy.concatenate(xs))
        self.original_targets.reset(numpy.concatenate(ts).astype(
            numpy.float32) / 255.0)
        self._apply_validation_ratio()

