"""Downloader, audio / text-stream loaders and the socket queue loader
(reference veles/downloader.py, loader/libsndfile_loader.py,
loader/hdfs_loader.py, zmq_loader.py)."""
import io
import os
import tarfile
import threading
import wave
import zipfile

import numpy
import pytest

from veles_amd.backends import Device
from veles_amd.downloader import Downloader, unpack
from veles_amd.dummy import DummyWorkflow
from veles_amd.error import BadFormatError
from veles_amd.loader.audio import (FullBatchAudioLoader, TextLinesLoader,
                                    decode_audio)
from veles_amd.loader.queue_loader import QueueLoader, QueueLoaderClient


def _wav(path, pcm, rate=8000, channels=1, width=2):
    with wave.open(str(path), "wb") as w:
        w.setnchannels(channels)
        w.setsampwidth(width)
        w.setframerate(rate)
        w.writeframes(pcm.tobytes())


def test_downloader_file_url_zip_and_skip(tmp_path):
    src = tmp_path / "src.zip"
    with zipfile.ZipFile(src, "w") as z:
        z.writestr("ds/a.txt", "hello")
    dst = tmp_path / "datasets"
    d = Downloader(DummyWorkflow(), url=src.as_uri(), files=["ds/a.txt"],
                   directory=str(dst))
    d.initialize()
    assert (dst / "ds" / "a.txt").read_text() == "hello"
    assert not (dst / "src.zip").exists()  # archive removed after unpack
    os.remove(src)  # present files: no second fetch
    d.initialize()


def test_downloader_missing_file_and_tar_escape(tmp_path):
    src = tmp_path / "x.tar.gz"
    with tarfile.open(src, "w:gz") as t:
        data = b"x"
        ti = tarfile.TarInfo("../evil.txt")
        ti.size = 1
        t.addfile(ti, io.BytesIO(data))
    with pytest.raises(ValueError):
        unpack(str(src), str(tmp_path / "out"))
    ok = tmp_path / "ok.tar"
    with tarfile.open(ok, "w") as t:
        ti = tarfile.TarInfo("b.txt")
        ti.size = 1
        t.addfile(ti, io.BytesIO(b"y"))
    d = Downloader(DummyWorkflow(), url=str(ok), files=["c.txt"],
                   directory=str(tmp_path / "o2"))
    with pytest.raises(FileNotFoundError):
        d.initialize()


def test_unpack_rejects_symlink_chain(tmp_path):
    """d/l -> .., d/l/m -> .., d/l/m/escaped.txt: every member passes a
    realpath check taken before extraction, yet the file lands two levels
    above the target.  Links are refused outright."""
    src = tmp_path / "chain.tar"
    with tarfile.open(src, "w") as t:
        for name in ("d/l", "d/l/m"):
            ti = tarfile.TarInfo(name)
            ti.type = tarfile.SYMTYPE
            ti.linkname = ".."
            t.addfile(ti)
        ti = tarfile.TarInfo("d/l/m/escaped.txt")
        ti.size = 1
        t.addfile(ti, io.BytesIO(b"z"))
    out = tmp_path / "a" / "b" / "out"
    out.mkdir(parents=True)
    with pytest.raises(ValueError):
        unpack(str(src), str(out))
    assert not list(tmp_path.rglob("escaped.txt"))
    hard = tmp_path / "hard.tar"
    with tarfile.open(hard, "w") as t:
        ti = tarfile.TarInfo("h")
        ti.type = tarfile.LNKTYPE
        ti.linkname = "../../etc/passwd"
        t.addfile(ti)
    with pytest.raises(ValueError):
        unpack(str(hard), str(out))


def test_decode_audio_widths(tmp_path):
    pcm = (numpy.arange(-50, 50, dtype=numpy.int16) * 300)
    _wav(tmp_path / "a.wav", pcm)
    d = decode_audio(str(tmp_path / "a.wav"))
    assert d["channels"] == 1 and d["samples"] == 100
    numpy.testing.assert_array_equal(d["data"], pcm)
    st = numpy.stack([pcm, -pcm], 1).astype(numpy.int16)
    _wav(tmp_path / "s.wav", st, channels=2)
    d = decode_audio(str(tmp_path / "s.wav"))
    numpy.testing.assert_array_equal(d["data"].reshape(-1, 2), st)
    u8 = (numpy.arange(0, 256, 2)).astype(numpy.uint8)
    _wav(tmp_path / "u.wav", u8, width=1)
    d = decode_audio(str(tmp_path / "u.wav"))
    numpy.testing.assert_array_equal(d["data"],
                                     (u8.astype(numpy.int16) - 128) << 8)
    (tmp_path / "bad.wav").write_bytes(b"not a wave file at all")
    with pytest.raises(BadFormatError):
        decode_audio(str(tmp_path / "bad.wav"))


def test_full_batch_audio_loader(tmp_path):
    rs = numpy.random.RandomState(0)
    for c in ("yes", "no"):
        os.makedirs(tmp_path / c)
        for i in range(3):
            n = 50 + 10 * i
            _wav(tmp_path / c / ("%d.wav" % i),
                 (rs.randn(n) * 1000).astype(numpy.int16))
    ld = FullBatchAudioLoader(DummyWorkflow(), train_paths=[str(tmp_path)],
                              samples=64, channels=2, minibatch_size=2)
    ld.initialize(device=Device(backend="cpu"))
    x = ld.original_data.mem
    assert x.shape == (6, 64, 2)
    assert numpy.abs(x).max() < 1.0
    assert (x[0, 50:] == 0).all()  # zero padded past the clip
    numpy.testing.assert_array_equal(x[..., 0], x[..., 1])  # mono -> stereo
    assert ld.reversed_labels_mapping == ["no", "yes"]
    assert sorted(ld.original_labels.tolist()) == [0, 0, 0, 1, 1, 1]


def test_text_lines_loader(tmp_path):
    f1, f2 = tmp_path / "a.txt", tmp_path / "b.txt"
    f1.write_text("l0\nl1\nl2\n")
    f2.write_text("l3\nl4\n")
    ld = TextLinesLoader(DummyWorkflow(), file=[str(f1), str(f2)], chunk=2)
    ld.initialize()
    got = []
    while not ld.finished:
        ld.run()
        got.extend(ld.output)
    assert got == ["l0", "l1", "l2", "l3", "l4"]


@pytest.mark.parametrize("transport", ["tcp", "ipc"])
def test_queue_loader_request_reply(transport):
    wf = DummyWorkflow()
    ql = QueueLoader(wf, transport=transport,
                     reply_fn=lambda w: {"sum": float(ql.output.sum())})
    ql.initialize()
    assert "QueueLoaderEndpoints" in ql.generate_data_for_master()
    cl = QueueLoaderClient(ql.endpoints)
    cl.send(numpy.arange(4, dtype=numpy.float32))
    ql.run()  # receives the first request
    numpy.testing.assert_array_equal(ql.output, [0, 1, 2, 3])
    cl.send(numpy.ones(3))
    ql.run()  # replies to the first, receives the second
    assert cl.receive() == {"sum": 6.0}
    t = threading.Thread(target=ql.run)  # replies, then blocks
    t.start()
    assert cl.receive() == {"sum": 3.0}
    ql.stop()  # unblocks the pending run() with None
    t.join(10)
    assert not t.is_alive() and ql.output is None
    cl.close()


def test_module_object_helpers():
    import veles_amd
    loc = veles_amd.__loc__
    assert loc["python"] > 1000 and loc["hip"] > 1000
    names = {u.__name__ for u in veles_amd.__units__}
    assert {"Downloader", "QueueLoader", "FullBatchAudioLoader",
            "All2All"} <= names
    assert isinstance(veles_amd.validate_environment(), list)
    veles_amd.check_root(allow=True)
    assert isinstance(veles_amd.__plugins__, set)
