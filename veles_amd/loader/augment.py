"""Geometric augmentation of the image loaders: which crop, mirror and
rotation each served sample gets.

Reference semantics (veles/loader/image.py:124-311, 516-568): ``crop`` =
(height, width) in pixels (int) or as a fraction of the canvas (float);
``crop_number`` crops per image and epoch; ``mirror`` False / True (every
image served twice, plain and flipped) / "random"; ``rotations`` a sorted
tuple of angles in radians, each image served once per angle;
``samples_inflation`` = (2 if mirror is True) * len(rotations) *
crop_number index slots per image; ``smart_crop`` keeps the crop window
overlapping the image's bounding box (``bbox`` = (ymin, ymax, xmin, xmax)).

MI355X design: the host only DRAWS the per-sample parameters from the
loader's PRNG (so ``-r`` seeds reproduce every crop and mirror), as a
float32 [B][6] table {cy, cx, cos, sin, mirror, 0}; the pixels are produced
on the device by ``ops.image_batch`` (hvk_image_batch), which also fuses
the Sobel channel, the background fill and the normalisation.  No
device->host synchronisation is involved.
"""
from __future__ import annotations

import math

import numpy

__all__ = ["Augmentation"]


class Augmentation(object):
    def __init__(self, crop=None, crop_number=1, mirror=False,
                 rotations=(0.0,), smart_crop=True, add_sobel=False):
        if crop is not None:
            crop = tuple(crop)
            if len(crop) != 2:
                raise ValueError("crop must be (height, width), got %r" %
                                 (crop,))
            for v in crop:
                if isinstance(v, bool) or not isinstance(v, (int, float)):
                    raise TypeError("crop entries must be int or float")
                if isinstance(v, int) and v < 1:
                    raise ValueError("crop %r out of range" % (crop,))
                if isinstance(v, float) and not 0 < v <= 1:
                    raise ValueError("fractional crop %r out of (0, 1]" %
                                     (crop,))
        if isinstance(crop_number, bool) or not isinstance(crop_number, int) \
                or crop_number < 1:
            raise ValueError("crop_number must be an integer >= 1")
        if crop_number > 1 and crop is None:
            raise ValueError("crop_number > 1 needs crop")
        if mirror not in (False, True, "random"):
            raise ValueError('mirror must be False, True or "random"')
        rotations = tuple(sorted(float(r) for r in rotations))
        if not rotations:
            raise ValueError("rotations must not be empty")
        if any(abs(r) >= 2 * math.pi for r in rotations):
            raise ValueError("rotations are radians in (-2 pi, 2 pi)")
        self.crop = crop
        self.crop_number = crop_number
        self.mirror = mirror
        self.rotations = rotations
        self.smart_crop = bool(smart_crop)
        self.add_sobel = bool(add_sobel)

    @property
    def samples_inflation(self):
        return (2 if self.mirror is True else 1) * len(self.rotations) * \
            self.crop_number

    @property
    def is_identity(self):
        return self.crop is None and self.mirror is False and \
            self.rotations == (0.0,) and not self.add_sobel

    def output_hw(self, canvas_hw):
        """(height, width) of a served sample cut from a canvas."""
        H, W = canvas_hw
        if self.crop is None:
            return H, W
        out = []
        for v, n in zip(self.crop, (H, W)):
            c = v if isinstance(v, int) else max(1, int(v * n))
            if c > n:
                raise ValueError("crop %r exceeds the canvas %s" %
                                 (self.crop, canvas_hw))
            out.append(c)
        return tuple(out)

    def channels(self, c):
        return c + (1 if self.add_sobel else 0)

    def distortion(self, dist_index, prng):
        """(mirror, angle) of distortion slot ``dist_index`` of an image
        (reference get_distortion_by_index)."""
        i = dist_index // self.crop_number
        if self.mirror is True:
            return bool(i % 2), self.rotations[i // 2]
        if self.mirror == "random":
            return bool(prng.randint(2)), self.rotations[i]
        return False, self.rotations[i]

    def params(self, canvas_hw, dist_indices, prng, bboxes=None,
               center=False):
        """float32 [B][6] parameters of ``ops.image_batch`` for samples with
        these distortion slots; ``bboxes`` [(ymin, ymax, xmin, xmax)] per
        sample (smart crop), ``center`` = deterministic centred crops and
        no random mirror (analysis passes)."""
        H, W = canvas_hw
        ch, cw = self.output_hw(canvas_hw)
        n = len(dist_indices)
        out = numpy.zeros((n, 6), numpy.float32)
        for b, d in enumerate(dist_indices):
            if center:
                mir, ang = False, 0.0
                cy, cx = (H - ch) // 2, (W - cw) // 2
            else:
                mir, ang = self.distortion(int(d), prng)
                cy = cx = 0
                if self.crop is not None:
                    bb = bboxes[b] if (bboxes is not None and
                                       self.smart_crop) else (0, H, 0, W)
                    # windows that overlap the box, inside the canvas
                    lo_y = max(int(bb[0]) - ch, 0)
                    hi_y = min(H - ch + 1, int(bb[1]) + ch)
                    lo_x = max(int(bb[2]) - cw, 0)
                    hi_x = min(W - cw + 1, int(bb[3]) + cw)
                    cy = int(prng.randint(lo_y, max(hi_y, lo_y + 1)))
                    cx = int(prng.randint(lo_x, max(hi_x, lo_x + 1)))
            out[b] = (cy, cx, math.cos(ang), math.sin(ang),
                      1.0 if mir else 0.0, 0.0)
        return out
