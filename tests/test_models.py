"""Wire contracts: protobuf schema, pinned enum numerics, S3 key layout."""
from __future__ import annotations

import base64
import os
import re

import pytest

from downloader_amd.models import api, keys


def test_pinned_status_numerics():
    assert api.string_to_enum("TelemetryStatusEntry", "DOWNLOADING") == 2
    assert api.string_to_enum("TelemetryStatusEntry", "ERRORED") == 6


def test_source_type_names_lowercase_to_methods():
    names = {api.enum_to_string("SourceType", v).lower() for v in api.ENUMS["SourceType"].values()}
    assert names == {"torrent", "http", "file", "bucket"}


def test_download_roundtrip_and_convert_copies_media():
    d = api.make_download("id1", "http", "http://x/y.mkv", "TV", creator_id="card9", name="Show")
    d2 = api.decode(api.Download, api.encode(d))
    assert d2.media.id == "id1" and d2.media.creatorId == "card9"
    assert d2.media.source == api.string_to_enum("SourceType", "HTTP")
    c = api.make_convert(d2.media)
    c2 = api.decode(api.Convert, api.encode(c))
    assert c2.media == d2.media
    assert re.fullmatch(r"\d{4}-\d\d-\d\dT\d\d:\d\d:\d\d\.\d{3}Z", c2.createdAt)


def test_proto_file_matches_runtime_schema():
    text = open(os.path.join(os.path.dirname(api.__file__), "api.proto")).read()
    for m, fields in api.MESSAGES.items():
        assert f"message {m} " in text
        for fname, num, _ in fields:
            assert re.search(rf"\b{fname} = {num};", text), (m, fname)
    for e, vals in api.ENUMS.items():
        for n, v in vals.items():
            assert f"{n} = {v};" in text


@pytest.mark.parametrize("parts,want", [
    (("a", "original/", "b"), "a/original/b"),
    (("a", "original/", "/b"), "a/original/b"),
    (("a", "original/", "b//c"), "a/original/b/c"),
    (("a", "original/", "b/"), "a/original/b/"),
    (("a/./x/..", "original/", "b"), "a/original/b"),
    (("", "x"), "x"),
])
def test_node_join(parts, want):
    assert keys.node_join(*parts) == want


def test_object_key_base64_layout():
    assert keys.object_key("m1", "/d/blob.mkv") == "m1/original/" + base64.b64encode(b"blob.mkv").decode()
    assert keys.done_key("m1") == "m1/original/done"
    assert keys.STAGING_BUCKET == "triton-staging"


def test_object_key_slash_in_base64_makes_segments():
    # App. A #10: '/' inside standard base64 creates key segments (and '//' collapses).
    name = next(n for n in (f"f{i}?.mkv" for i in range(2000))
                if "/" in base64.b64encode(n.encode()).decode())
    b64 = base64.b64encode(name.encode()).decode()
    k = keys.object_key("id", "/x/" + name)
    assert k == keys.node_normalize("id/original/" + b64)
    assert k.count("/") >= 3


def test_enum_to_string_invalid():
    with pytest.raises(ValueError):
        api.enum_to_string("SourceType", 99)
