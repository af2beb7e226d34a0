"""Audio and text-stream loaders.

* ``decode_audio`` / ``FullBatchAudioLoader`` replace the reference's
  libsndfile ctypes loaders (veles/loader/libsndfile.py,
  veles/loader/libsndfile_loader.py:46-108: decode to signed 16-bit PCM,
  mono or stereo only).  libsndfile is not part of this image, so decoding
  uses the stdlib ``wave`` module (PCM WAV, 8/16/24/32-bit); other formats
  raise ``BadFormatError`` like the reference's failed ``sf_open``.  Clips
  are cut / zero-padded to ``samples`` frames and served as float features
  in [-1, 1) through the full-batch device gather.
* ``TextLinesLoader`` replaces ``HDFSTextLoader``
  (veles/loader/hdfs_loader.py:48-71): it streams ``chunk`` lines per run
  from local (or mounted HDFS) text files and raises ``finished`` at the end.
"""
from __future__ import annotations

import io
import wave

import numpy

from veles_amd.distributable import TriviallyDistributable
from veles_amd.error import BadFormatError
from veles_amd.loader.base import TEST, TRAIN, VALID
from veles_amd.loader.file_loader import FileFilter, label_from_path, \
    scan_files
from veles_amd.loader.fullbatch import FullBatchLoader
from veles_amd.mutable import Bool
from veles_amd.units import Unit

__all__ = ["decode_audio", "FullBatchAudioLoader", "TextLinesLoader",
           "AUDIO_TYPES"]

AUDIO_TYPES = ("wav", "wave")


def decode_audio(path_or_bytes):
    """-> dict(data=int16[frames * channels] interleaved, sampling_rate,
    samples, channels, name)."""
    name = path_or_bytes if isinstance(path_or_bytes, str) else "<bytes>"
    src = io.BytesIO(path_or_bytes) if isinstance(
        path_or_bytes, (bytes, bytearray)) else path_or_bytes
    try:
        w = wave.open(src, "rb")
    except (wave.Error, EOFError) as e:
        raise BadFormatError("%s: unsupported audio format (%s)" % (name, e))
    with w:
        ch, width, rate, n = (w.getnchannels(), w.getsampwidth(),
                              w.getframerate(), w.getnframes())
        if ch > 2:
            raise BadFormatError("%s has %d channels; only mono or stereo "
                                 "are allowed" % (name, ch))
        raw = w.readframes(n)
    if width == 1:
        pcm = (numpy.frombuffer(raw, numpy.uint8).astype(numpy.int16) - 128) \
            << 8
    elif width == 2:
        pcm = numpy.frombuffer(raw, "<i2").astype(numpy.int16)
    elif width == 3:
        b = numpy.frombuffer(raw, numpy.uint8).reshape(-1, 3)
        pcm = (b[:, 2].astype(numpy.int8).astype(numpy.int16) << 8) | b[:, 1]
    elif width == 4:
        pcm = (numpy.frombuffer(raw, "<i4") >> 16).astype(numpy.int16)
    else:
        raise BadFormatError("%s: %d-byte samples" % (name, width))
    return {"data": numpy.ascontiguousarray(pcm), "sampling_rate": rate,
            "samples": n, "channels": ch, "name": name}


class FullBatchAudioLoader(FullBatchLoader):
    """Audio clips from ``train_paths`` / ``validation_paths`` /
    ``test_paths`` (files or directories); the label is the parent directory
    name or ``label_regexp``'s group.  Each sample is ``samples`` frames x
    ``channels`` (mono clips are duplicated when ``channels`` is 2)."""
    MAPPING = "full_batch_audio"

    def __init__(self, workflow, **kwargs):
        super().__init__(workflow, **kwargs)
        self.paths = {TEST: list(kwargs.get("test_paths", ())),
                      VALID: list(kwargs.get("validation_paths", ())),
                      TRAIN: list(kwargs.get("train_paths", ()))}
        self.samples = int(kwargs.get("samples", 16000))
        self.channels = int(kwargs.get("channels", 1))
        self.label_regexp = kwargs.get("label_regexp")
        self.filter = FileFilter(mime_types=(), filename_types=kwargs.get(
            "file_subtypes", AUDIO_TYPES))

    def _clip(self, d):
        pcm = d["data"].reshape(-1, d["channels"])
        if d["channels"] < self.channels:
            pcm = numpy.repeat(pcm, self.channels, axis=1)
        elif d["channels"] > self.channels:
            pcm = pcm.mean(axis=1, keepdims=True).astype(numpy.int16)
        out = numpy.zeros((self.samples, self.channels), numpy.float32)
        n = min(self.samples, len(pcm))
        out[:n] = pcm[:n] / 32768.0
        return out

    def load_data(self):
        datas, labels = [], []
        self.class_lengths = [0, 0, 0]
        for cls in (TEST, VALID, TRAIN):
            for f in scan_files(self.paths[cls], self.filter):
                datas.append(self._clip(decode_audio(f)))
                labels.append(label_from_path(f, self.label_regexp))
                self.class_lengths[cls] += 1
        if not datas:
            raise BadFormatError("no audio files found in %s" % self.paths)
        self.original_data.reset(numpy.stack(datas))
        names = sorted(set(labels))
        self.labels_mapping = {v: i for i, v in enumerate(names)}
        self.reversed_labels_mapping = names
        self.original_labels = numpy.array(
            [self.labels_mapping[v] for v in labels], numpy.int32)
        self._apply_validation_ratio()


class TextLinesLoader(Unit, TriviallyDistributable):
    """``file``: one path or a list; ``chunk``: lines per run.  ``output``
    holds the chunk (short at the end); ``finished`` turns True after the
    last line was served."""

    def __init__(self, workflow, **kwargs):
        kwargs.setdefault("view_group", "LOADER")
        super().__init__(workflow, **kwargs)
        f = kwargs["file"]
        self.file_names = [f] if isinstance(f, str) else list(f)
        self.chunk_lines_number = int(kwargs.get("chunk", 1000))
        self.encoding = kwargs.get("encoding", "utf-8")
        self.output = []
        self.finished = Bool(False)

    def init_unpickled(self):
        super().init_unpickled()
        self._generator_ = None

    def _lines(self):
        for fn in self.file_names:
            with open(fn, encoding=self.encoding) as f:
                for line in f:
                    yield line.rstrip("\n")

    def initialize(self, **kwargs):
        self._generator_ = self._lines()
        self.finished <<= False

    def run(self):
        assert not self.finished, "TextLinesLoader ran after the last line"
        out = []
        for line in self._generator_:
            out.append(line)
            if len(out) == self.chunk_lines_number:
                break
        else:
            self.finished <<= True
        self.output = out
