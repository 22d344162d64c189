"""AMQP 0-9-1 wire codec (frames, method arguments, field tables, basic properties).

Shared by the client (``broker.amqp``) and the bundled broker (``broker.server``). Covers the
classes the staging service needs: connection, channel, queue, basic and confirm.
"""
from __future__ import annotations

import struct
from dataclasses import dataclass, field
from decimal import Decimal
from typing import Any, Dict, List, Optional, Tuple

PROTOCOL_HEADER = b"AMQP\x00\x00\x09\x01"
FRAME_METHOD, FRAME_HEADER, FRAME_BODY, FRAME_HEARTBEAT = 1, 2, 3, 8
FRAME_END = 0xCE
FRAME_MIN = 4096

# (class, method) ids
CONNECTION_START = (10, 10)
CONNECTION_START_OK = (10, 11)
CONNECTION_TUNE = (10, 30)
CONNECTION_TUNE_OK = (10, 31)
CONNECTION_OPEN = (10, 40)
CONNECTION_OPEN_OK = (10, 41)
CONNECTION_CLOSE = (10, 50)
CONNECTION_CLOSE_OK = (10, 51)
CHANNEL_OPEN = (20, 10)
CHANNEL_OPEN_OK = (20, 11)
CHANNEL_FLOW = (20, 20)
CHANNEL_FLOW_OK = (20, 21)
CHANNEL_CLOSE = (20, 40)
CHANNEL_CLOSE_OK = (20, 41)
QUEUE_DECLARE = (50, 10)
QUEUE_DECLARE_OK = (50, 11)
QUEUE_PURGE = (50, 30)
QUEUE_PURGE_OK = (50, 31)
QUEUE_DELETE = (50, 40)
QUEUE_DELETE_OK = (50, 41)
BASIC_QOS = (60, 10)
BASIC_QOS_OK = (60, 11)
BASIC_CONSUME = (60, 20)
BASIC_CONSUME_OK = (60, 21)
BASIC_CANCEL = (60, 30)
BASIC_CANCEL_OK = (60, 31)
BASIC_PUBLISH = (60, 40)
BASIC_RETURN = (60, 50)
BASIC_DELIVER = (60, 60)
BASIC_GET = (60, 70)
BASIC_GET_OK = (60, 71)
BASIC_GET_EMPTY = (60, 72)
BASIC_ACK = (60, 80)
BASIC_REJECT = (60, 90)
BASIC_RECOVER = (60, 110)
BASIC_RECOVER_OK = (60, 111)
BASIC_NACK = (60, 120)
CONFIRM_SELECT = (85, 10)
CONFIRM_SELECT_OK = (85, 11)

# Argument signatures: o=octet s=short l=long L=longlong S=shortstr T=longstr F=table b=bit
SIGNATURES: Dict[Tuple[int, int], str] = {
    CONNECTION_START: "ooFTT",
    CONNECTION_START_OK: "FSTS",
    CONNECTION_TUNE: "sls",
    CONNECTION_TUNE_OK: "sls",
    CONNECTION_OPEN: "SSb",
    CONNECTION_OPEN_OK: "S",
    CONNECTION_CLOSE: "sSss",
    CONNECTION_CLOSE_OK: "",
    CHANNEL_OPEN: "S",
    CHANNEL_OPEN_OK: "T",
    CHANNEL_FLOW: "b",
    CHANNEL_FLOW_OK: "b",
    CHANNEL_CLOSE: "sSss",
    CHANNEL_CLOSE_OK: "",
    QUEUE_DECLARE: "sSbbbbbF",
    QUEUE_DECLARE_OK: "Sll",
    QUEUE_PURGE: "sSb",
    QUEUE_PURGE_OK: "l",
    QUEUE_DELETE: "sSbbb",
    QUEUE_DELETE_OK: "l",
    BASIC_QOS: "lsb",
    BASIC_QOS_OK: "",
    BASIC_CONSUME: "sSSbbbbF",
    BASIC_CONSUME_OK: "S",
    BASIC_CANCEL: "Sb",
    BASIC_CANCEL_OK: "S",
    BASIC_PUBLISH: "sSSbb",
    BASIC_RETURN: "sSSS",
    BASIC_DELIVER: "SLbSS",
    BASIC_GET: "sSb",
    BASIC_GET_OK: "LbSSl",
    BASIC_GET_EMPTY: "S",
    BASIC_ACK: "Lb",
    BASIC_REJECT: "Lb",
    BASIC_RECOVER: "b",
    BASIC_RECOVER_OK: "",
    BASIC_NACK: "Lbb",
    CONFIRM_SELECT: "b",
    CONFIRM_SELECT_OK: "",
}

# methods that carry content (header + body frames follow)
CONTENT_METHODS = {BASIC_PUBLISH, BASIC_DELIVER, BASIC_GET_OK, BASIC_RETURN}


class AMQPError(Exception):
    def __init__(self, msg: str, code: int = 0):
        super().__init__(msg)
        self.code = code


class FrameError(AMQPError):
    pass


# ---------------------------------------------------------------- primitive encoders
def enc_shortstr(s) -> bytes:
    b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
    if len(b) > 255:
        raise AMQPError("shortstr too long")
    return bytes([len(b)]) + b


def enc_longstr(s) -> bytes:
    b = s.encode("utf-8") if isinstance(s, str) else bytes(s)
    return struct.pack(">I", len(b)) + b


def enc_value(v: Any) -> bytes:
    if isinstance(v, bool):
        return b"t" + (b"\x01" if v else b"\x00")
    if isinstance(v, int):
        return b"l" + struct.pack(">q", v)
    if isinstance(v, float):
        return b"d" + struct.pack(">d", v)
    if isinstance(v, Decimal):
        sign, digits, exp = v.as_tuple()
        iv = int("".join(map(str, digits)) or "0") * (-1 if sign else 1)
        return b"D" + struct.pack(">Bi", max(0, -exp), iv)
    if isinstance(v, str):
        return b"S" + enc_longstr(v)
    if isinstance(v, (bytes, bytearray)):
        return b"x" + enc_longstr(bytes(v))
    if isinstance(v, dict):
        return b"F" + enc_table(v)
    if isinstance(v, (list, tuple)):
        body = b"".join(enc_value(x) for x in v)
        return b"A" + struct.pack(">I", len(body)) + body
    if v is None:
        return b"V"
    raise AMQPError(f"cannot encode field value of type {type(v).__name__}")


def enc_table(d: Optional[Dict[str, Any]]) -> bytes:
    if not d:
        return b"\x00\x00\x00\x00"
    body = b"".join(enc_shortstr(k) + enc_value(v) for k, v in d.items())
    return struct.pack(">I", len(body)) + body


class Reader:
    __slots__ = ("b", "i", "bitbyte", "bitpos")

    def __init__(self, b: bytes, i: int = 0):
        self.b = b
        self.i = i
        self.bitbyte = 0
        self.bitpos = 8

    def _take(self, n: int) -> bytes:
        if self.i + n > len(self.b):
            raise FrameError("truncated frame payload")
        v = self.b[self.i:self.i + n]
        self.i += n
        return v

    def octet(self) -> int:
        self.bitpos = 8
        return self._take(1)[0]

    def short(self) -> int:
        self.bitpos = 8
        return struct.unpack(">H", self._take(2))[0]

    def long(self) -> int:
        self.bitpos = 8
        return struct.unpack(">I", self._take(4))[0]

    def longlong(self) -> int:
        self.bitpos = 8
        return struct.unpack(">Q", self._take(8))[0]

    def shortstr(self) -> str:
        self.bitpos = 8
        n = self._take(1)[0]
        return self._take(n).decode("utf-8", "replace")

    def longstr(self) -> bytes:
        self.bitpos = 8
        n = struct.unpack(">I", self._take(4))[0]
        return self._take(n)

    def bit(self) -> bool:
        if self.bitpos >= 8:
            self.bitbyte = self._take(1)[0]
            self.bitpos = 0
        v = bool(self.bitbyte & (1 << self.bitpos))
        self.bitpos += 1
        return v

    def table(self) -> Dict[str, Any]:
        self.bitpos = 8
        n = struct.unpack(">I", self._take(4))[0]
        end = self.i + n
        out: Dict[str, Any] = {}
        while self.i < end:
            k = self.shortstr()
            out[k] = self.value()
        return out

    def value(self) -> Any:
        t = self._take(1)
        if t == b"t":
            return bool(self._take(1)[0])
        if t == b"b":
            return struct.unpack(">b", self._take(1))[0]
        if t == b"B":
            return self._take(1)[0]
        if t in (b"s", b"U"):
            return struct.unpack(">h", self._take(2))[0]
        if t == b"u":
            return struct.unpack(">H", self._take(2))[0]
        if t == b"I":
            return struct.unpack(">i", self._take(4))[0]
        if t == b"i":
            return struct.unpack(">I", self._take(4))[0]
        if t in (b"l", b"L"):
            return struct.unpack(">q", self._take(8))[0]
        if t == b"f":
            return struct.unpack(">f", self._take(4))[0]
        if t == b"d":
            return struct.unpack(">d", self._take(8))[0]
        if t == b"D":
            scale, iv = struct.unpack(">Bi", self._take(5))
            return Decimal(iv).scaleb(-scale)
        if t == b"S":
            return self.longstr().decode("utf-8", "replace")
        if t == b"x":
            return self.longstr()
        if t == b"A":
            n = struct.unpack(">I", self._take(4))[0]
            end = self.i + n
            arr = []
            while self.i < end:
                arr.append(self.value())
            return arr
        if t == b"T":
            return struct.unpack(">Q", self._take(8))[0]
        if t == b"F":
            return self.table()
        if t == b"V":
            return None
        raise FrameError(f"unknown field type {t!r}")


def encode_args(sig: str, args: List[Any]) -> bytes:
    out = bytearray()
    bits: List[bool] = []

    def flush() -> None:
        if bits:
            for i in range(0, len(bits), 8):
                byte = 0
                for j, b in enumerate(bits[i:i + 8]):
                    if b:
                        byte |= 1 << j
                out.append(byte)
            bits.clear()

    if len(args) != len(sig):
        raise AMQPError(f"expected {len(sig)} args, got {len(args)}")
    for t, v in zip(sig, args):
        if t == "b":
            bits.append(bool(v))
            continue
        flush()
        if t == "o":
            out += struct.pack(">B", v)
        elif t == "s":
            out += struct.pack(">H", v)
        elif t == "l":
            out += struct.pack(">I", v)
        elif t == "L":
            out += struct.pack(">Q", v)
        elif t == "S":
            out += enc_shortstr(v)
        elif t == "T":
            out += enc_longstr(v)
        elif t == "F":
            out += enc_table(v)
    flush()
    return bytes(out)


def decode_args(sig: str, r: Reader) -> List[Any]:
    out: List[Any] = []
    for t in sig:
        if t == "o":
            out.append(r.octet())
        elif t == "s":
            out.append(r.short())
        elif t == "l":
            out.append(r.long())
        elif t == "L":
            out.append(r.longlong())
        elif t == "S":
            out.append(r.shortstr())
        elif t == "T":
            out.append(r.longstr())
        elif t == "F":
            out.append(r.table())
        elif t == "b":
            out.append(r.bit())
    return out


def method_frame(channel: int, method: Tuple[int, int], *args: Any) -> bytes:
    payload = struct.pack(">HH", *method) + encode_args(SIGNATURES[method], list(args))
    return struct.pack(">BHI", FRAME_METHOD, channel, len(payload)) + payload + bytes([FRAME_END])


_MALFORMED = (struct.error, IndexError, KeyError, ValueError, UnicodeDecodeError,
              OverflowError, TypeError)


def decode_method(payload: bytes) -> Tuple[Tuple[int, int], List[Any]]:
    """Method frame payload -> ((class, method), args). Any malformed payload is a
    FrameError (the connection's read loop treats it as a broken connection)."""
    try:
        cid, mid = struct.unpack(">HH", payload[:4])
        m = (cid, mid)
        sig = SIGNATURES.get(m)
        if sig is None:
            raise FrameError(f"unsupported method {m}")
        return m, decode_args(sig, Reader(payload, 4))
    except _MALFORMED as e:
        raise FrameError(f"malformed method frame: {type(e).__name__}: {e}") from e


# ---------------------------------------------------------------- content
@dataclass
class Properties:
    content_type: Optional[str] = None
    content_encoding: Optional[str] = None
    headers: Dict[str, Any] = field(default_factory=dict)
    delivery_mode: Optional[int] = None
    priority: Optional[int] = None
    correlation_id: Optional[str] = None
    reply_to: Optional[str] = None
    expiration: Optional[str] = None
    message_id: Optional[str] = None
    timestamp: Optional[int] = None
    type: Optional[str] = None
    user_id: Optional[str] = None
    app_id: Optional[str] = None

    _ORDER = ("content_type", "content_encoding", "headers", "delivery_mode", "priority",
              "correlation_id", "reply_to", "expiration", "message_id", "timestamp", "type",
              "user_id", "app_id")
    _KIND = ("S", "S", "F", "o", "o", "S", "S", "S", "S", "L", "S", "S", "S")

    def encode(self) -> bytes:
        flags = 0
        body = bytearray()
        for i, (name, kind) in enumerate(zip(self._ORDER, self._KIND)):
            v = getattr(self, name)
            if v is None or (name == "headers" and not v):
                continue
            flags |= 1 << (15 - i)
            body += encode_args(kind, [v])
        return struct.pack(">H", flags) + bytes(body)

    @classmethod
    def decode(cls, r: Reader) -> "Properties":
        flags = r.short()
        p = cls()
        for i, (name, kind) in enumerate(zip(cls._ORDER, cls._KIND)):
            if flags & (1 << (15 - i)):
                setattr(p, name, decode_args(kind, r)[0])
        return p


def header_frame(channel: int, body_size: int, props: Properties, class_id: int = 60) -> bytes:
    payload = struct.pack(">HHQ", class_id, 0, body_size) + props.encode()
    return struct.pack(">BHI", FRAME_HEADER, channel, len(payload)) + payload + bytes([FRAME_END])


def decode_header(payload: bytes) -> Tuple[int, Properties]:
    try:
        r = Reader(payload)
        r.short()  # class id
        r.short()  # weight
        size = r.longlong()
        return size, Properties.decode(r)
    except _MALFORMED as e:
        raise FrameError(f"malformed content header: {type(e).__name__}: {e}") from e


def body_frames(channel: int, body: bytes, frame_max: int) -> List[bytes]:
    step = max(1, frame_max - 8)
    return [struct.pack(">BHI", FRAME_BODY, channel, len(body[i:i + step])) + body[i:i + step]
            + bytes([FRAME_END]) for i in range(0, len(body), step)]


def heartbeat_frame() -> bytes:
    return struct.pack(">BHI", FRAME_HEARTBEAT, 0, 0) + bytes([FRAME_END])


async def read_frame(reader) -> Tuple[int, int, bytes]:
    hdr = await reader.readexactly(7)
    ftype, ch, size = struct.unpack(">BHI", hdr)
    if size > 128 << 20:
        raise FrameError("frame too large")
    payload = await reader.readexactly(size + 1)
    if payload[-1] != FRAME_END:
        raise FrameError("bad frame end")
    return ftype, ch, payload[:-1]


def content_frames(channel: int, method_bytes: bytes, body: bytes, props: Properties,
                   frame_max: int) -> bytes:
    return method_bytes + header_frame(channel, len(body), props) + b"".join(
        body_frames(channel, body, frame_max))
