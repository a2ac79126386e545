"""fqz5file._Sink on outputs that cannot take positioned writes:
a FIFO (as a pipe or /dev/stdout is) gets the decoded text sequentially,
writes that arrive ahead of the stream held until the gap before them is
written; a regular file keeps positioned writes."""
import os
import threading

import pytest

from fqzcomp5_amd.fqz5file import _Sink


def test_sink_fifo_in_order(tmp_path):
    p = str(tmp_path / "f")
    os.mkfifo(p)
    got = []
    t = threading.Thread(target=lambda: got.append(open(p, "rb").read()))
    t.start()
    s = _Sink(p, True)
    assert s.seq
    s.write_at(5, b"world")          # ahead of the stream: held
    s.write_at(0, b"hello")
    s.write_at(10, memoryview(b"!!"))
    s.close()
    t.join(10)
    assert got == [b"helloworld!!"]


def test_sink_fifo_gap_is_an_error(tmp_path):
    p = str(tmp_path / "f")
    os.mkfifo(p)
    t = threading.Thread(target=lambda: open(p, "rb").read())
    t.start()
    s = _Sink(p, True)
    s.write_at(3, b"abc")
    with pytest.raises(ValueError):
        s.close()
    t.join(10)


def test_sink_regular_file_positioned(tmp_path):
    p = str(tmp_path / "r")
    s = _Sink(p, True)
    assert not s.seq
    s.write_at(4, b"5678")
    s.write_at(0, b"1234")
    s.close()
    assert open(p, "rb").read() == b"12345678"
