"""The swarm's GPU mode sizes its host-hashed tail by the download rate and the device's
measured per-piece latency (torrent/session.py ``_tail_due``): the last
pieces of a torrent are hashed on the host once what is left would download in less than the
device's submission -> digest time, so that time no longer lands on the end of the job."""
from __future__ import annotations

from types import SimpleNamespace

from downloader_amd.torrent import session as sess


class _Wire:
    def __init__(self, lat: float):
        self.rx = 0
        self.lat = lat

    def rx_total(self) -> int:
        return self.rx

    def gpu_latency(self) -> float:
        return self.lat


def _session(total: int, lat: float, auto: bool = True, fixed: int = 0):
    return SimpleNamespace(wire=_Wire(lat), _tail_auto=auto,
                           client=SimpleNamespace(swarm_gpu_tail_x=1.3),
                           _tail_bytes=total // 2 if auto else fixed,
                           _tail_t=0.0, _tail_rx0=None)


def test_auto_tail_follows_rate_and_latency(monkeypatch):
    clock = [100.0]
    monkeypatch.setattr(sess.time, "monotonic", lambda: clock[0])
    s = _session(16 << 30, lat=0.1)
    due = lambda left: sess.TorrentSession._tail_due(s, left)   # noqa: E731
    assert not due(8 << 30)                 # no byte received yet: no rate
    clock[0] += 0.01
    s.wire.rx = 1 << 20
    assert not due(8 << 30)                 # first byte: the rate's origin
    clock[0] += 0.05
    s.wire.rx += int(0.5e9)                 # 10 GB/s since the first byte
    # tail = 10 GB/s x 0.1 s x 1.3 = 1.3 GB
    assert not due(2 << 30)
    clock[0] += 0.01
    s.wire.rx += int(0.1e9)
    assert due(1 << 30)


def test_auto_tail_is_checked_at_most_every_5_ms_and_capped_at_half(monkeypatch):
    clock = [10.0]
    monkeypatch.setattr(sess.time, "monotonic", lambda: clock[0])
    s = _session(1 << 30, lat=5.0)          # a device far slower than the download
    s.wire.rx = 1
    assert not sess.TorrentSession._tail_due(s, 900 << 20)
    clock[0] += 0.03
    s.wire.rx += 300 << 20
    # rate x latency is huge, but the tail is at most half the torrent
    assert not sess.TorrentSession._tail_due(s, 600 << 20)
    clock[0] += 0.001                       # within 5 ms of the last check: not re-evaluated
    assert not sess.TorrentSession._tail_due(s, 400 << 20)
    clock[0] += 0.01
    assert sess.TorrentSession._tail_due(s, 500 << 20)


def test_latency_default_before_the_first_digest_and_fixed_tail(monkeypatch):
    clock = [50.0]
    monkeypatch.setattr(sess.time, "monotonic", lambda: clock[0])
    s = _session(8 << 30, lat=0.0)          # no device digest yet: 0.12 s assumed
    s.wire.rx = 1
    sess.TorrentSession._tail_due(s, 4 << 30)
    clock[0] += 0.1
    s.wire.rx += int(1e9)                   # 10 GB/s -> tail 10 x 0.12 x 1.3 = 1.56 GB
    assert not sess.TorrentSession._tail_due(s, 1700 << 20)
    clock[0] += 0.01
    assert sess.TorrentSession._tail_due(s, 1300 << 20)   # 9.1 GB/s by now: 1.42 GB
    fixed = _session(8 << 30, lat=0.0, auto=False, fixed=256 << 20)
    assert not sess.TorrentSession._tail_due(fixed, 300 << 20)
    assert sess.TorrentSession._tail_due(fixed, 256 << 20)
