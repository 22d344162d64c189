"""Protobuf wire models for package ``api`` (the reference's ``triton-core/proto``).

The reference decodes ``api.Download`` from ``v1.download`` (lib/main.js:63), encodes
``api.Convert`` onto ``v1.convert`` (lib/main.js:157-164) and maps enum names with
``proto.stringToEnum`` / ``proto.enumToString`` (lib/download.js:32,243, lib/upload.js:16,
lib/process.js:53). ``protoc`` is not installed, so the descriptor is assembled here from
the same schema as ``api.proto`` and classes are produced by the protobuf runtime.
"""
from __future__ import annotations

import datetime as _dt
from typing import Any, Dict, Type

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory
from google.protobuf import json_format

_F = descriptor_pb2.FieldDescriptorProto

ENUMS: Dict[str, Dict[str, int]] = {
    "SourceType": {"TORRENT": 0, "HTTP": 1, "FILE": 2, "BUCKET": 3},
    "MediaType": {"MOVIE": 0, "TV": 1},
    "TelemetryStatusEntry": {
        "QUEUED": 0, "METADATA": 1, "DOWNLOADING": 2, "CONVERTING": 3,
        "UPLOADING": 4, "DEPLOYED": 5, "ERRORED": 6,
    },
    "CreatorType": {"API": 0, "TRELLO": 1},
}

# (name, number, scalar-type | ('enum', Name) | ('msg', Name))
MESSAGES = {
    "Media": [
        ("id", 1, _F.TYPE_STRING), ("name", 2, _F.TYPE_STRING),
        ("creator", 3, ("enum", "CreatorType")), ("creatorId", 4, _F.TYPE_STRING),
        ("type", 5, ("enum", "MediaType")), ("source", 6, ("enum", "SourceType")),
        ("sourceURI", 7, _F.TYPE_STRING), ("metadataId", 8, _F.TYPE_STRING),
        ("status", 9, ("enum", "TelemetryStatusEntry")),
    ],
    "Download": [("createdAt", 1, _F.TYPE_STRING), ("media", 2, ("msg", "Media"))],
    "Convert": [("createdAt", 1, _F.TYPE_STRING), ("media", 2, ("msg", "Media"))],
    "TelemetryStatus": [
        ("mediaId", 1, _F.TYPE_STRING), ("status", 2, ("enum", "TelemetryStatusEntry")),
    ],
    "TelemetryProgress": [
        ("mediaId", 1, _F.TYPE_STRING), ("status", 2, ("enum", "TelemetryStatusEntry")),
        ("progress", 3, _F.TYPE_INT32),
    ],
}


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fdp = descriptor_pb2.FileDescriptorProto(name="downloader_amd/api.proto", package="api",
                                             syntax="proto3")
    for ename, values in ENUMS.items():
        e = fdp.enum_type.add(name=ename)
        for vname, num in values.items():
            e.value.add(name=vname, number=num)
    for mname, fields in MESSAGES.items():
        m = fdp.message_type.add(name=mname)
        for fname, num, ftype in fields:
            f = m.field.add(name=fname, number=num, label=_F.LABEL_OPTIONAL, json_name=fname)
            if isinstance(ftype, tuple):
                kind, ref = ftype
                f.type = _F.TYPE_ENUM if kind == "enum" else _F.TYPE_MESSAGE
                f.type_name = ".api." + ref
            else:
                f.type = ftype
    return fdp


_POOL = descriptor_pool.DescriptorPool()
_POOL.Add(_build_file())

Media: Type[Any] = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("api.Media"))
Download: Type[Any] = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("api.Download"))
Convert: Type[Any] = message_factory.GetMessageClass(_POOL.FindMessageTypeByName("api.Convert"))
TelemetryStatus: Type[Any] = message_factory.GetMessageClass(
    _POOL.FindMessageTypeByName("api.TelemetryStatus"))
TelemetryProgress: Type[Any] = message_factory.GetMessageClass(
    _POOL.FindMessageTypeByName("api.TelemetryProgress"))

TYPES = {"api.Media": Media, "api.Download": Download, "api.Convert": Convert,
         "api.TelemetryStatus": TelemetryStatus, "api.TelemetryProgress": TelemetryProgress}

# Pinned numerics the reference hard-codes (lib/main.js:68,149).
STATUS_DOWNLOADING = ENUMS["TelemetryStatusEntry"]["DOWNLOADING"]
STATUS_ERRORED = ENUMS["TelemetryStatusEntry"]["ERRORED"]
assert STATUS_DOWNLOADING == 2 and STATUS_ERRORED == 6


def load(name: str) -> Type[Any]:
    """``proto.load('api.X')`` equivalent (reference lib/main.js:55)."""
    try:
        return TYPES[name]
    except KeyError:
        raise KeyError(f"unknown message type {name!r}") from None


def string_to_enum(enum: str, key: str) -> int:
    """``proto.stringToEnum(type, enum, key)`` (reference lib/download.js:32)."""
    return ENUMS[enum][key]


def enum_to_string(enum: str, value: int) -> str:
    """``proto.enumToString(type, enum, int)`` (reference lib/download.js:243)."""
    for k, v in ENUMS[enum].items():
        if v == value:
            return k
    raise ValueError(f"{value} is not a valid {enum}")


def encode(msg: Any) -> bytes:
    return msg.SerializeToString()


def decode(cls: Type[Any], data: bytes) -> Any:
    m = cls()
    m.ParseFromString(bytes(data))
    return m


def to_dict(msg: Any) -> Dict[str, Any]:
    return json_format.MessageToDict(msg, preserving_proto_field_name=True,
                                     always_print_fields_with_no_presence=True)


def now_iso() -> str:
    """ISO-8601 UTC timestamp with millisecond precision and ``Z`` suffix, matching
    JavaScript ``new Date().toISOString()`` (reference lib/main.js:158)."""
    t = _dt.datetime.now(_dt.timezone.utc)
    return t.strftime("%Y-%m-%dT%H:%M:%S.") + f"{t.microsecond // 1000:03d}Z"


def make_convert(media: Any) -> Any:
    """Build the ``api.Convert`` follow-up job; media is copied verbatim (lib/main.js:157-160)."""
    c = Convert(createdAt=now_iso())
    c.media.CopyFrom(media)
    return c


def make_download(media_id: str, source: str, uri: str, media_type: str = "MOVIE",
                  creator_id: str = "", name: str = "") -> Any:
    d = Download(createdAt=now_iso())
    d.media.id = media_id
    d.media.name = name
    d.media.creatorId = creator_id
    d.media.source = string_to_enum("SourceType", source.upper())
    d.media.sourceURI = uri
    d.media.type = string_to_enum("MediaType", media_type.upper())
    return d
