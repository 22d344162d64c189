"""Prometheus metrics (the reference's ``triton-core/prom``).

The reference creates ``Prom.new('downloader')`` and calls ``Prom.expose()`` (lib/main.js:43-44)
but defines no service metrics of its own. Here each worker owns a registry with the
staging metrics listed in SURVEY.md §5.5; the bench harness reads them back.
"""
from __future__ import annotations

import time
from contextlib import contextmanager
from typing import Iterator, Optional

from prometheus_client import (CollectorRegistry, Counter, Gauge, Histogram,
                               generate_latest, start_http_server)
from prometheus_client import CONTENT_TYPE_LATEST  # noqa: F401

_BUCKETS = (0.005, 0.01, 0.025, 0.05, 0.1, 0.25, 0.5, 1, 2.5, 5, 10, 30, 60, 120, 300, 900, 3600)


class _RuntimeCollector:
    def __init__(self, transports, ns: str):
        self.transports = transports
        self.ns = ns

    def describe(self):
        return []

    def collect(self):
        from prometheus_client.core import CounterMetricFamily, GaugeMetricFamily
        nt = getattr(self.transports, "native", None)
        if nt is not None:
            yield GaugeMetricFamily(f"{self.ns}_http_idle_connections",
                                    "idle keep-alive connections of the native transport",
                                    value=nt.idle_connections())
        try:
            from ..ops import native
            st = native().relay_pool_stats()
        except Exception:     # extension not built: nothing to report
            return
        yield GaugeMetricFamily(f"{self.ns}_relay_pool_in_use",
                                "relay part buffers in use", value=st["in_use"])
        yield GaugeMetricFamily(f"{self.ns}_relay_pool_idle_bytes",
                                "bytes held by idle relay part buffers", value=st["idle_bytes"])
        yield GaugeMetricFamily(f"{self.ns}_relay_pool_in_use_bytes",
                                "bytes of leased relay part buffers", value=st["in_use_bytes"])
        yield GaugeMetricFamily(f"{self.ns}_relay_pool_budget_bytes",
                                "part-buffer budget (leased + idle never exceed it; 0 = none)",
                                value=st["budget"])
        yield GaugeMetricFamily(f"{self.ns}_relay_pool_peak_bytes",
                                "high-water mark of leased + idle part buffers",
                                value=st["peak_bytes"])
        # > 0 means a lease was granted past the budget (a part larger than the whole budget)
        yield CounterMetricFamily(f"{self.ns}_relay_pool_over_budget",
                                  "part-buffer leases granted past the budget",
                                  value=st["over_budget"])
        gs = native().gpu_part_stats()
        yield GaugeMetricFamily(f"{self.ns}_gpu_parts_pending",
                                "relayed parts handed to the GPU hasher, not yet finished",
                                value=gs["pending"])
        yield CounterMetricFamily(f"{self.ns}_gpu_parts_submitted",
                                  "relayed parts handed to the GPU hasher",
                                  value=gs["submitted"])
        yield CounterMetricFamily(f"{self.ns}_gpu_parts_host_fallbacks",
                                  "GPU-queued parts hashed on the host (device failed before "
                                  "the DMA ended)", value=gs["host_fallbacks"])
        ps = native().pipe_stats()
        yield GaugeMetricFamily(f"{self.ns}_splice_pipes_in_use",
                                "splice pipes leased by running transfers", value=ps["in_use"])
        # a growing count means the uid's pipe page budget (fs.pipe-user-pages-soft) is spent:
        # pipes come out smaller than asked, or transfers copy through user space instead
        yield CounterMetricFamily(f"{self.ns}_splice_pipes_short",
                                  "splice pipes created below the asked capacity",
                                  value=ps["short"])


class Metrics:
    def __init__(self, namespace: str = "downloader", registry: Optional[CollectorRegistry] = None):
        self.registry = registry or CollectorRegistry(auto_describe=True)
        ns = namespace
        r = self.registry
        self.bytes_downloaded = Counter("bytes_downloaded_total", "bytes fetched from sources",
                                        ["proto"], namespace=ns, registry=r)
        self.bytes_uploaded = Counter("bytes_uploaded_total", "bytes uploaded to staging",
                                      namespace=ns, registry=r)
        self.bytes_verified = Counter("bytes_verified_total", "bytes piece-hash verified",
                                      ["backend"], namespace=ns, registry=r)
        self.job_duration = Histogram("job_duration_seconds", "end-to-end job latency",
                                      ["outcome"], namespace=ns, registry=r, buckets=_BUCKETS)
        self.stage_duration = Histogram("stage_duration_seconds", "per-stage latency",
                                        ["stage"], namespace=ns, registry=r, buckets=_BUCKETS)
        self.inflight = Gauge("inflight_jobs", "jobs currently being processed",
                              namespace=ns, registry=r)
        self.jobs = Counter("jobs_total", "jobs by outcome", ["outcome"], namespace=ns, registry=r)
        self.stalls = Counter("stall_total", "download stalls", namespace=ns, registry=r)
        self.retries = Counter("retries_total", "job redeliveries scheduled", namespace=ns,
                               registry=r)
        self.key_collisions = Counter("key_collisions_total",
                                      "files whose staging key collided within a job",
                                      namespace=ns, registry=r)
        self.telemetry_events = Counter("telemetry_events_total",
                                        "telemetry events by fate (published, dropped from "
                                        "the full outbox, failed publish attempts)",
                                        ["outcome"], namespace=ns, registry=r)
        self.telemetry_buffered = Gauge("telemetry_buffered",
                                        "telemetry events waiting in the outbox",
                                        namespace=ns, registry=r)
        self.messages = Counter("broker_messages_total", "broker traffic", ["queue", "op"],
                                namespace=ns, registry=r)
        self.stale_uploads = Counter("stale_uploads_aborted_total",
                                     "multipart uploads left open by earlier attempts, aborted "
                                     "when their job ended", namespace=ns, registry=r)

    def watch_runtime(self, transports=None, namespace: str = "downloader") -> None:
        """Gauges read at scrape time from the native runtime: idle keep-alive connections
        of the native transport and the hashed relay's part-buffer pool (in use / idle
        bytes). Registered once per registry."""
        if getattr(self, "_runtime", None) is not None:
            return
        self._runtime = _RuntimeCollector(transports, namespace)
        self.registry.register(self._runtime)

    @contextmanager
    def time_stage(self, stage: str) -> Iterator[None]:
        t0 = time.perf_counter()
        try:
            yield
        finally:
            self.stage_duration.labels(stage).observe(time.perf_counter() - t0)

    def exposition(self) -> bytes:
        return generate_latest(self.registry)

    def expose(self, port: int, addr: str = "0.0.0.0") -> None:
        """``Prom.expose()`` equivalent: serve /metrics on a dedicated port."""
        start_http_server(port, addr=addr, registry=self.registry)

    def sample(self, name: str, **labels: str) -> float:
        v = self.registry.get_sample_value(name, labels or None)
        return 0.0 if v is None else v
