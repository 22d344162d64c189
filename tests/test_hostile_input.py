"""Property tests: bytes from the network (peers, trackers, .torrent URLs, magnets, the
broker) are hostile. Each decoder either returns a value or raises its own error type - no
IndexError / KeyError / struct.error / RecursionError escapes into the worker."""
from __future__ import annotations

import hashlib

import pytest
from hypothesis import HealthCheck, given, settings
from hypothesis import strategies as st

from downloader_amd.broker import amqp_codec as C
from downloader_amd.torrent.bencode import BencodeError, bdecode, bencode, decode_torrent
from downloader_amd.torrent.magnet import MagnetError, parse_magnet
from downloader_amd.torrent.metainfo import MetainfoError, parse_info, parse_torrent

SETTINGS = settings(max_examples=300, deadline=None,
                    suppress_health_check=[HealthCheck.too_slow])


@SETTINGS
@given(st.binary(max_size=400))
def test_bdecode_only_raises_bencode_error(data):
    try:
        bdecode(data)
    except BencodeError:
        pass


def test_bdecode_deep_nesting_is_an_error_not_a_crash():
    with pytest.raises(BencodeError):
        bdecode(b"l" * 100_000 + b"e" * 100_000)


_VALID = bencode({b"announce": b"http://t/a", b"info": {
    b"name": b"x.mkv", b"piece length": 16384, b"length": 40000,
    b"pieces": hashlib.sha1(b"a").digest() * 3}})


@SETTINGS
@given(st.lists(st.tuples(st.integers(0, len(_VALID) - 1), st.integers(0, 255)),
                min_size=1, max_size=6))
def test_mutated_torrent_only_raises_metainfo_error(muts):
    data = bytearray(_VALID)
    for i, v in muts:
        data[i] = v
    try:
        m = parse_torrent(bytes(data))
    except MetainfoError:
        return
    assert m.num_pieces * m.piece_length >= m.total_length


@SETTINGS
@given(st.binary(max_size=300))
def test_info_dict_from_peers_only_raises_metainfo_error(data):
    try:
        parse_info(data)
    except MetainfoError:
        pass


@SETTINGS
@given(st.text(max_size=200))
def test_magnet_only_raises_magnet_error(s):
    for uri in (s, "magnet:?" + s, "magnet:?xt=urn:btih:" + s):
        try:
            parse_magnet(uri)
        except MagnetError:
            pass


@SETTINGS
@given(st.binary(max_size=300))
def test_amqp_method_and_header_decoding_only_raise_amqp_errors(payload):
    for fn in (C.decode_method, C.decode_header):
        try:
            fn(payload)
        except C.AMQPError:
            pass


@SETTINGS
@given(st.binary(max_size=200))
def test_torrent_span_finder_only_raises_bencode_error(data):
    try:
        decode_torrent(b"d4:info" + data)
    except BencodeError:
        pass


def test_broker_survives_garbage_frames(run):
    """A client that sends malformed frames loses its own connection; the bundled broker
    keeps serving everyone else."""
    import asyncio
    import struct

    from downloader_amd.broker.amqp import AmqpBroker
    from downloader_amd.broker.server import BrokerServer

    async def go():
        srv = await BrokerServer().start()
        host, port = "127.0.0.1", int(srv.url.rsplit(":", 1)[1].split("/")[0])
        for junk in (b"\x01\x00\x00\x00\x00\x00\x03\xff\xff\xff\xce",
                     b"AMQP\x00\x00\x09\x01" + b"\x01\x00\x00\x00\x00\x00\x02\x00" + b"\xce",
                     b"\x00" * 64):
            r, w = await asyncio.open_connection(host, port)
            w.write(junk if junk.startswith(b"AMQP") else b"AMQP\x00\x00\x09\x01" + junk)
            await w.drain()
            try:
                await asyncio.wait_for(r.read(1 << 16), 2)
            except asyncio.TimeoutError:
                pass
            w.close()
        b = AmqpBroker(srv.url)
        await b.connect()
        await b.declare("q")
        await b.publish("q", struct.pack(">I", 7))
        d = await b.get("q")
        assert d is not None and d.body == struct.pack(">I", 7)
        await d.ack()
        await b.close()
        await srv.stop()
    run(go())


_TRK = st.recursive(
    st.one_of(st.integers(-5, 10**6), st.binary(max_size=40)),
    lambda ch: st.one_of(st.lists(ch, max_size=3),
                         st.dictionaries(st.sampled_from([b"peers", b"ip", b"port", b"interval",
                                                          b"failure reason", b"peers6",
                                                          b"complete", b"x"]), ch, max_size=4)),
    max_leaves=10)


@SETTINGS
@given(_TRK)
def test_tracker_response_only_raises_tracker_error(v):
    from downloader_amd.torrent.tracker import TrackerError, parse_announce_response
    try:
        r = parse_announce_response(bencode(v))
    except TrackerError:
        return
    assert all(isinstance(h, str) and isinstance(p, int) for h, p in r.peers)
