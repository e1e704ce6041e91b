"""L0 utilities vs the reference's util/*.go semantics."""
import io

import pytest

from arena_amd.utils import (TabWriter, parse_data_dir_raw, parse_duration, random_int32,
                             retry_during, short_human_duration, validate_datasets,
                             validate_job_name)
from arena_amd.utils.errors import NEED_WAIT, is_retryable
from arena_amd.utils.validate import ValidationError
from arena_amd.version import semver


@pytest.mark.parametrize("name,ok", [("tf-git", True), ("a", True), ("a" * 63, True),
                                      ("a" * 64, False), ("Tf", False), ("-a", False),
                                      ("a-", False), ("a.b", False), ("a_b", False), ("", False)])
def test_validate_job_name(name, ok):
    if ok:
        validate_job_name(name)
    else:
        with pytest.raises(ValidationError):
            validate_job_name(name)


def test_job_name_message_says_63():  # Q13
    with pytest.raises(ValidationError, match="less than 63"):
        validate_job_name("a" * 70)


@pytest.mark.parametrize("ds,ok", [(["data:/data"], True), (["d:/data"], False),
                                    (["data:/"], False), (["data:rel"], False),
                                    (["nodest"], False), (["a:b:/c"], False),
                                    (["da$ta:/data"], False), (["my.data_1:/mnt/x"], True)])
def test_validate_datasets(ds, ok):
    if ok:
        validate_datasets(ds)
    else:
        with pytest.raises(ValidationError):
            validate_datasets(ds)


def test_parse_data_dir_raw():
    assert parse_data_dir_raw("/data") == ("/data", "/data")
    assert parse_data_dir_raw("/host/x:/ctr/y") == ("/host/x", "/ctr/y")
    for bad in ("/a:/b:/c", ":/x", "rel:/x", "/x:rel", "/", "/x:/"):
        with pytest.raises(ValidationError):
            parse_data_dir_raw(bad)


@pytest.mark.parametrize("secs,out", [(-5, "<invalid>"), (-0.5, "0s"), (0, "0s"), (59, "59s"),
                                       (60, "1m"), (3599, "59m"), (3600, "1h"),
                                       (86399, "23h"), (86400, "1d"), (86400 * 364, "364d"),
                                       (86400 * 365, "1y"), (86400 * 800, "2y")])
def test_short_human_duration(secs, out):
    assert short_human_duration(secs) == out


def test_parse_duration():
    assert parse_duration("5s") == 5
    assert parse_duration("2m") == 120
    assert parse_duration("3h") == 3 * 3600
    assert parse_duration("1h30m15s") == 5415
    assert parse_duration("300ms") == pytest.approx(0.3)
    assert parse_duration("42") == 42  # reference behaviour (integer seconds) still accepted
    with pytest.raises(ValueError):
        parse_duration("5x")


def test_random_int32_is_nine_digits():
    vals = {random_int32() for _ in range(50)}
    assert all(len(v) == 9 and v.isdigit() for v in vals)
    assert len(vals) > 40


def test_retry_during_classification():
    calls = {"n": 0}

    def cb():
        calls["n"] += 1
        if calls["n"] < 3:
            raise RuntimeError(NEED_WAIT)

    retry_during(10, 0, cb, sleep=lambda s: None)
    assert calls["n"] == 3
    with pytest.raises(ValueError):
        retry_during(10, 0, lambda: (_ for _ in ()).throw(ValueError("boom")), sleep=lambda s: None)
    t = {"now": 0.0}

    def clock():
        t["now"] += 5
        return t["now"]

    with pytest.raises(RuntimeError, match="attempts"):
        retry_during(12, 0, lambda: (_ for _ in ()).throw(RuntimeError("connection refused")),
                     clock=clock, sleep=lambda s: None)
    assert is_retryable("unexpected EOF")


def test_tabwriter_matches_go_layout():
    b = io.StringIO()
    w = TabWriter(b)
    w.write("NAME\tSTATUS\tTRAINER\tAGE\tNODE\n")
    w.write("tf-git\tRUNNING\tTFJOB\t5m\t192.168.1.1\n")
    w.flush()
    assert b.getvalue() == ("NAME    STATUS   TRAINER  AGE  NODE\n"
                            "tf-git  RUNNING  TFJOB    5m   192.168.1.1\n")


def test_semver():
    assert semver("v0.1.0", "abcdef123", "clean", "0.1.0") == "v0.1.0"
    assert semver("", "abcdef123", "clean", "0.1.0") == "v0.1.0+abcdef1"
    assert semver("v0.1.0", "abcdef123", "dirty", "0.1.0") == "v0.1.0+abcdef1.dirty"
    assert semver("", "", "", "0.1.0") == "v0.1.0+unknown"
