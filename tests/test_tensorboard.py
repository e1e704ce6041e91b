"""TensorBoard event files + the built-in scalar server (SURVEY §5 metrics row: the reference
hostPath-mounts a log dir for TensorBoard, charts/tfjob/templates/{deployment,service}.yaml).

The writer hand-encodes TFRecord + Event protobufs. Wire compatibility is checked against the
real protobuf runtime, decoding with a dynamically-built copy of TensorFlow's ``Event`` schema
(tensorflow/core/util/event.proto field numbers) -- tensorboard itself is not installed here.
"""
from __future__ import annotations

import json
import struct
import threading
import urllib.request
from http.server import ThreadingHTTPServer

import pytest

from arena_amd.tb import writer as W
from arena_amd.tb.server import make_handler


def test_crc32c_check_value():
    assert W.crc32c(b"123456789") == 0xE3069283          # RFC 3720 check value
    assert W.crc32c(b"") == 0


def _event_classes():
    pb = pytest.importorskip("google.protobuf")  # noqa: F841
    from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
    f = descriptor_pb2.FileDescriptorProto(name="ev_test.proto", package="t")
    val = f.message_type.add(name="Value")
    val.field.add(name="tag", number=1, type=9, label=1)
    val.field.add(name="simple_value", number=2, type=2, label=1)
    summ = f.message_type.add(name="Summary")
    summ.field.add(name="value", number=1, type=11, label=3, type_name=".t.Value")
    ev = f.message_type.add(name="Event")
    ev.field.add(name="wall_time", number=1, type=1, label=1)
    ev.field.add(name="step", number=2, type=3, label=1)
    ev.field.add(name="file_version", number=3, type=9, label=1)
    ev.field.add(name="summary", number=5, type=11, label=1, type_name=".t.Summary")
    pool = descriptor_pool.DescriptorPool()
    pool.Add(f)
    desc = pool.FindMessageTypeByName("t.Event")
    try:
        return message_factory.GetMessageClass(desc)
    except AttributeError:  # older protobuf
        return message_factory.MessageFactory(pool).GetPrototype(desc)


def _records(path):
    data = open(path, "rb").read()
    i, out = 0, []
    while i < len(data):
        (n,) = struct.unpack_from("<Q", data, i)
        (lcrc,) = struct.unpack_from("<I", data, i + 8)
        assert lcrc == W.masked_crc(data[i:i + 8])
        body = data[i + 12:i + 12 + n]
        (dcrc,) = struct.unpack_from("<I", data, i + 12 + n)
        assert dcrc == W.masked_crc(body)
        out.append(body)
        i += 16 + n
    return out


def test_event_file_is_valid_tfrecord_of_event_protos(tmp_path):
    Event = _event_classes()
    sw = W.SummaryWriter(str(tmp_path / "train"))
    for step in range(0, 50, 10):
        sw.add_scalar("accuracy", 0.9 + step / 1000, step)
    sw.add_scalars({"loss": 0.25, "lr": 1e-3}, 60)
    sw.close()
    recs = _records(sw.path)
    assert len(recs) == 7
    first = Event.FromString(recs[0])
    assert first.file_version == "brain.Event:2"
    e = Event.FromString(recs[3])
    assert e.step == 20 and e.summary.value[0].tag == "accuracy"
    assert e.summary.value[0].simple_value == pytest.approx(0.92, rel=1e-6)
    last = Event.FromString(recs[-1])
    assert {v.tag: round(v.simple_value, 6) for v in last.summary.value} == {"loss": 0.25,
                                                                            "lr": 0.001}
    # and our own reader agrees
    scal = W.read_scalars(str(tmp_path))
    assert [s for s, _ in scal["train"]["accuracy"]] == [0, 10, 20, 30, 40]
    assert scal["train"]["loss"][0][0] == 60


def test_scalar_server_serves_json_and_html(tmp_path):
    sw = W.SummaryWriter(str(tmp_path / "test"))
    sw.add_scalar("accuracy", 0.9649, 990)
    sw.close()
    srv = ThreadingHTTPServer(("127.0.0.1", 0), make_handler(str(tmp_path)))
    th = threading.Thread(target=srv.serve_forever, daemon=True)
    th.start()
    try:
        base = f"http://127.0.0.1:{srv.server_address[1]}"
        d = json.load(urllib.request.urlopen(base + "/data/scalars", timeout=10))
        assert d["test"]["accuracy"][0][0] == 990
        page = urllib.request.urlopen(base + "/", timeout=10).read().decode()
        assert "test / accuracy" in page and "<svg" in page and "0.9649" in page
    finally:
        srv.shutdown()
