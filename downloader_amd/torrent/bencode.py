"""Bencoding (BEP-3) - replaces the ``bencode@2`` package in the reference's webtorrent stack
(yarn.lock:336). Dict keys decode to ``bytes``; ``decode_torrent`` also returns the exact byte
span of the ``info`` dict so the infohash is computed over the original encoding."""
from __future__ import annotations

from typing import Any, Dict, List, Optional, Tuple, Union

Bencodable = Union[int, bytes, str, List[Any], Dict[Any, Any]]


class BencodeError(ValueError):
    pass


class _Decoder:
    __slots__ = ("d", "i", "info_span", "depth")

    def __init__(self, data: bytes):
        self.d = data
        self.i = 0
        self.info_span: Optional[Tuple[int, int]] = None
        self.depth = 0

    def value(self) -> Any:
        d, i = self.d, self.i
        if i >= len(d):
            raise BencodeError("unexpected end of data")
        c = d[i]
        if c == 0x69:  # i
            end = d.index(b"e", i + 1)
            raw = d[i + 1:end]
            if not raw or raw == b"-" or (raw.startswith(b"0") and len(raw) > 1) \
                    or raw.startswith(b"-0"):
                raise BencodeError(f"bad integer {raw!r}")
            self.i = end + 1
            return int(raw)
        if 0x30 <= c <= 0x39:
            colon = d.index(b":", i)
            n = int(d[i:colon])
            start = colon + 1
            if start + n > len(d):
                raise BencodeError("string overruns data")
            self.i = start + n
            return d[start:start + n]
        if c == 0x6C:  # l
            self.i += 1
            self.depth += 1
            if self.depth > 64:
                raise BencodeError("nesting too deep")
            out = []
            while True:
                if self.i >= len(d):
                    raise BencodeError("unterminated list")
                if d[self.i] == 0x65:
                    self.i += 1
                    self.depth -= 1
                    return out
                out.append(self.value())
        if c == 0x64:  # d
            self.i += 1
            self.depth += 1
            if self.depth > 64:
                raise BencodeError("nesting too deep")
            res: Dict[bytes, Any] = {}
            while True:
                if self.i >= len(d):
                    raise BencodeError("unterminated dict")
                if d[self.i] == 0x65:
                    self.i += 1
                    self.depth -= 1
                    return res
                k = self.value()
                if not isinstance(k, bytes):
                    raise BencodeError("dict key must be a string")
                vstart = self.i
                res[k] = self.value()
                if k == b"info" and self.depth == 1 and self.info_span is None:
                    self.info_span = (vstart, self.i)
        raise BencodeError(f"invalid token {chr(c)!r} at {i}")


def bdecode(data: bytes, strict_end: bool = True) -> Any:
    dec = _Decoder(bytes(data))
    try:
        v = dec.value()
    except (ValueError, IndexError) as e:
        if isinstance(e, BencodeError):
            raise
        raise BencodeError(str(e)) from e
    if strict_end and dec.i != len(dec.d):
        raise BencodeError("trailing data after bencoded value")
    return v


def bdecode_prefix(data: bytes) -> Tuple[Any, int]:
    """Decode one value at the start of ``data``; returns (value, bytes consumed). Used by
    ut_metadata where the raw metadata piece follows the bencoded header."""
    dec = _Decoder(bytes(data))
    try:
        v = dec.value()
    except (ValueError, IndexError) as e:
        raise BencodeError(str(e)) from e
    return v, dec.i


def decode_torrent(data: bytes) -> Tuple[Dict[bytes, Any], bytes]:
    dec = _Decoder(bytes(data))
    try:
        v = dec.value()
    except (ValueError, IndexError) as e:
        raise BencodeError(str(e)) from e
    if not isinstance(v, dict) or dec.info_span is None:
        raise BencodeError("torrent has no info dictionary")
    a, b = dec.info_span
    return v, dec.d[a:b]


def bencode(obj: Bencodable) -> bytes:
    out: List[bytes] = []
    _enc(obj, out)
    return b"".join(out)


def _enc(o: Any, out: List[bytes]) -> None:
    if isinstance(o, bool):
        raise TypeError("bool is not bencodable")
    if isinstance(o, int):
        out.append(b"i%de" % o)
    elif isinstance(o, (bytes, bytearray, memoryview)):
        b = bytes(o)
        out.append(b"%d:" % len(b))
        out.append(b)
    elif isinstance(o, str):
        b = o.encode("utf-8")
        out.append(b"%d:" % len(b))
        out.append(b)
    elif isinstance(o, (list, tuple)):
        out.append(b"l")
        for x in o:
            _enc(x, out)
        out.append(b"e")
    elif isinstance(o, dict):
        out.append(b"d")
        items = [(k.encode("utf-8") if isinstance(k, str) else bytes(k), v) for k, v in o.items()]
        for k, v in sorted(items, key=lambda kv: kv[0]):
            out.append(b"%d:" % len(k))
            out.append(k)
            _enc(v, out)
        out.append(b"e")
    else:
        raise TypeError(f"cannot bencode {type(o).__name__}")
