"""Service kernel / job orchestrator (reference lib/main.js:40-205).

Per delivery of ``v1.download`` (``processor``, lib/main.js:62-170):
  1. decode ``api.Download`` (:63), emit status DOWNLOADING=2 (:68), register the job (:70-73)
  2. idempotence guard: a staged ``<id>/original/done`` marker skips straight to 5 (:117-126)
  3. run the stages in order, each seeing ``lastStage`` (:127-140)
  4. failure policy (:141-151): ``ERRDLSTALL`` -> ack and drop; anything else -> status
     ERRORED=6 and retry (reference: ``nack``)
  5. publish ``api.Convert{createdAt, media}`` to ``v1.convert`` (:157-164), then ack (:168)

Fixes: only NoSuchKey/404 means "not staged" (#5); a failed convert publish
is nacked for redelivery instead of being left unacked (#8); the active-job registry really
removes finished jobs (#2), so ``/health`` and shutdown behave.

Retry policy (``broker.max_retries``, reference AMQP arg ``2`` INFERRED): a failed job is
re-published with ``x-attempt`` + 1 after exponential backoff, then dead-lettered to
``broker.dead_letter_queue`` when the budget is spent. The backoff is held by the broker (a
TTL holding queue dead-lettering back to ``v1.download``), not by this consumer: the failed
delivery is acked at once, so its prefetch slot goes to the next job. ``mode: reference``
uses plain ``nack(requeue)``.
"""
from __future__ import annotations

import asyncio
import time
from collections import deque
from dataclasses import dataclass, field
from typing import Any, Deque, Dict, List, Optional, Tuple

from ..broker.base import Broker, Delivery, make_broker
from ..models import api, keys
from ..net.http import TransportSet, make_transports
from ..s3.client import S3Client, S3Error
from ..stages import build_stages
from ..stages.base import EventEmitter, Job, Services, Stage
from ..stages.jobdir import get_reaper
from ..utils import limits
from ..utils.config import Config
from ..utils.log import Logger, get_logger, redact_text
from ..utils.metrics import Metrics
from ..utils.trace import Tracer, init_tracer
from .telemetry import Telemetry


@dataclass
class ActiveJob:
    job_id: str
    creator_id: str
    started: float = field(default_factory=time.time)
    stage: str = ""


@dataclass
class JobResult:
    job_id: str
    outcome: str            # staged | skipped | stalled | retried | dead | failed | publish_failed
    seconds: float
    bytes: int = 0
    error: str = ""
    stats: dict = field(default_factory=dict)   # the job's stats (stage timings, torrent, ...)


RESULTS_MAX = 10_000


def _attempt(headers: Dict[str, Any]) -> int:
    """``x-attempt`` of a delivery. Headers come from whoever published the message: a value
    that is not a small non-negative integer counts as attempt 0 instead of raising before
    the delivery is acked or nacked (which would leave it stuck unacked)."""
    try:
        return max(0, min(1 << 20, int(headers.get("x-attempt", 0) or 0)))
    except (TypeError, ValueError, OverflowError):
        return 0


class Worker:
    def __init__(self, cfg: Config, broker: Optional[Broker] = None,
                 s3: Optional[S3Client] = None, transports: Optional[TransportSet] = None,
                 telemetry: Optional[Telemetry] = None, metrics: Optional[Metrics] = None,
                 tracer: Optional[Tracer] = None, logger: Optional[Logger] = None):
        self.cfg = cfg
        self.log = logger or get_logger("main")
        self.metrics = metrics or Metrics()
        self.broker = broker or make_broker(cfg, self.metrics)
        self.transports = transports or make_transports(
            native=cfg.s3.native_transport or cfg.download.http_native,
            max_workers=max(16, cfg.concurrency * 2 *
                            (cfg.s3.max_inflight_parts + cfg.download.http_streams)),
            connect_timeout=cfg.s3.connect_timeout_s, io_timeout=cfg.s3.request_timeout_s,
            ssl_verify=cfg.tls.verify, ca_file=cfg.tls.ca_file, native_tls=cfg.tls.native)
        self.s3 = s3 or S3Client.from_config(cfg.s3, self.transports)
        self.metrics.watch_runtime(self.transports)
        self.telemetry = telemetry or Telemetry.from_config(cfg, self.broker, self.log,
                                                            self.metrics)
        self.tracer = tracer or init_tracer("downloader", cfg.trace.enabled, cfg.trace.path)
        self.services = Services(cfg, self.telemetry, self.s3, self.transports, self.metrics,
                                 self.tracer, self.log)
        self.stages: List[Tuple[str, Stage]] = []
        self.active: Dict[int, ActiveJob] = {}
        # most recent outcomes (tests, bench, debugging); bounded for long-running workers
        self.results: Deque[JobResult] = deque(maxlen=RESULTS_MAX)
        self._consumer: Optional[str] = None
        self._inflight: set = set()
        self._stopping = False
        self._health = None
        self._seq = 0
        self.on_result = None  # optional callback(JobResult)

    # ------------------------------------------------------------------ lifecycle
    async def init(self) -> None:
        """Connect and build stages without consuming (used by tests and the bench)."""
        await self.broker.connect()
        await self.telemetry.connect()
        for q in (self.cfg.broker.download_queue, self.cfg.broker.convert_queue,
                  self.cfg.broker.dead_letter_queue):
            await self.broker.declare(q)
        if not self.stages:
            self.stages = await build_stages(self.cfg.stages, self.cfg, self.services)
        get_reaper(self.services).sweep()   # trash left by a crashed predecessor
        d = self.cfg.download
        # the uid's pipe page budget is shared: size splice pipes to this worker's share
        self.pipe_bytes = limits.apply_pipe_size(d.pipe_kb, d.pipe_sharers)
        if d.gpu_prewarm and d.stream_verify_backend == "gpu" and d.stream_gpu_pending > 0:
            await self._prewarm_part_hasher()
        # (auto sets the PartHasher up on an executor thread when a job first wants it - a
        # worker that never stages a big webseed torrent never initialises HIP)
        if d.gpu_prewarm and d.verify_backend != "cpu":
            from ..ops import hashing
            # auto never picks the GPU on a host with the multi-buffer SHA-1: no HIP init
            if d.verify_backend == "auto" and not hashing.auto_may_use_gpu():
                return
            prewarm_gpu = hashing.prewarm_gpu
            try:
                warm = await asyncio.get_running_loop().run_in_executor(None, prewarm_gpu)
                self.log.info({"gpu_verifier": warm}, "gpu verifier prewarm")
            except Exception as e:  # a missing device must not stop the worker
                self.log.warn({"err": str(e)}, "gpu verifier prewarm failed")

    async def _prewarm_part_hasher(self) -> None:
        """stream_verify_backend gpu: set up the gfx950 PartHasher now (HIP init and device
        slots, off the event loop) instead of inside the first job. (``auto`` starts the same
        set-up in the background when a job first wants it: torrent.stream.start_gpu_init.)"""
        from ..ops import gpu_available, hashing
        d = self.cfg.download
        loop = asyncio.get_running_loop()
        try:
            if not await loop.run_in_executor(None, gpu_available):
                return
            ok = await loop.run_in_executor(
                None, lambda: hashing.gpu_relay_hashing(
                    d.stream_gpu_min_pieces, d.stream_gpu_slots, d.stream_gpu_slot_mb << 20,
                    copy_streams=d.stream_gpu_copy_streams,
                    compute_streams=d.stream_gpu_compute_streams))
            self.log.info({"gpu_part_hasher": ok}, "gpu relay hashing prewarm")
        except Exception as e:  # a broken device must not stop the worker
            self.log.warn({"err": str(e)}, "gpu relay hashing prewarm failed")

    async def start(self, health: bool = True) -> None:
        await self.init()
        self._consumer = await self.broker.consume(self.cfg.broker.download_queue,
                                                   self._on_delivery, self.cfg.broker.prefetch)
        if health and self.cfg.health.enabled:
            from .health import HealthServer
            self._health = HealthServer(self, self.cfg.health)
            await self._health.start()
        if self.cfg.metrics.enabled and self.cfg.metrics.port:
            self.metrics.expose(self.cfg.metrics.port)
        self.log.info("successfully connected to queue and started server")

    async def stop(self, drain_timeout: float = 30.0) -> int:
        """Stop consuming, let in-flight jobs finish (bounded), close everything.
        Returns the process exit code the reference's termHandler would use (lib/main.js:197-204):
        0 when nothing was in flight, 1 otherwise."""
        self._stopping = True
        had_active = bool(self.active)
        if self._consumer is not None:
            try:
                await self.broker.cancel(self._consumer)
            except Exception:
                pass
            self._consumer = None
        if self._inflight:
            await asyncio.wait(list(self._inflight), timeout=drain_timeout)
        if self._health is not None:
            await self._health.stop()
        for _, st in self.stages:
            await st.close()
        await asyncio.get_running_loop().run_in_executor(None, get_reaper(self.services).close,
                                                         drain_timeout)
        # events of the drained jobs: flushed while the broker takes them (bounded)
        await self.telemetry.close(timeout=2 * self.cfg.telemetry.publish_timeout_s)
        try:
            await self.broker.close()
        except Exception:
            pass
        await self.s3.close()
        await self.transports.close()
        self.tracer.close()             # drains the span exporter thread
        return 1 if had_active and self.active else 0

    # ------------------------------------------------------------------ message path
    async def _on_delivery(self, d: Delivery) -> None:
        t = asyncio.current_task()
        self._inflight.add(t)
        try:
            await self.process(d)
        finally:
            self._inflight.discard(t)

    async def process(self, d: Delivery) -> JobResult:
        t0 = time.perf_counter()
        try:
            msg = api.decode(api.Download, d.body)
        except Exception as e:
            self.log.error("undecodable message dropped to dead-letter", err=str(e))
            await self._dead_letter(d, f"decode: {e}")
            return self._finish(None, JobResult("", "dead", time.perf_counter() - t0, error=str(e)))
        media = msg.media
        job_id, creator = media.id, media.creatorId
        attempt = _attempt(d.headers)
        child = self.log.child(jobId=job_id, fileId=creator)
        self._seq += 1
        slot = self._seq
        self.active[slot] = ActiveJob(job_id, creator)
        self.metrics.inflight.inc()
        await self.telemetry.emit_status(job_id, api.STATUS_DOWNLOADING)
        emitter = EventEmitter()
        job = Job(msg=msg, media=media, logger=child, emitter=emitter, attempt=attempt,
                  headers=dict(d.headers))
        outcome, err = "staged", ""
        try:
            with self.tracer.span("job", traceparent=d.headers.get("traceparent"),
                                  job_id=job_id, attempt=attempt) as span:
                staged = await self._already_staged(job_id, child)
                if not staged:
                    child.info("starting main processor after successful stage init")
                    try:
                        await self._run_stages(job, slot)
                    except Exception as e:
                        code = getattr(e, "code", None)
                        child.error("failed to invoke stage:", str(e))
                        if code == "ERRDLSTALL":
                            self.metrics.stalls.inc()
                            if self.cfg.download.emit_errored_on_stall:
                                await self.telemetry.emit_status(job_id, api.STATUS_ERRORED)
                            await d.ack()
                            return self._finish(job, JobResult(job_id, "stalled",
                                                          time.perf_counter() - t0, error=str(e)))
                        await self.telemetry.emit_status(job_id, api.STATUS_ERRORED)
                        outcome = await self._retry(d, attempt, str(e))
                        if outcome == "dead":
                            await self._sweep_uploads(job, child)
                        return self._finish(job, JobResult(job_id, outcome, time.perf_counter() - t0,
                                                      error=str(e)))
                    child.info("creating convert job")
                    if attempt > 0 or d.redelivered:
                        # an earlier attempt may have left uploads open (killed worker, kept
                        # resumable relay that this attempt did not need)
                        await self._sweep_uploads(job, child)
                else:
                    outcome = "skipped"
                    child.warn("skipping download due to files existing in triton-staging")
                try:
                    conv = api.make_convert(media)
                    hdrs = {"traceparent": span.traceparent()}
                    await self.broker.publish(self.cfg.broker.convert_queue, api.encode(conv), hdrs)
                    self.metrics.messages.labels(self.cfg.broker.convert_queue, "publish").inc()
                except Exception as e:
                    child.error("failed to create job:", str(e))
                    await d.nack(requeue=True)
                    return self._finish(job, JobResult(job_id, "publish_failed",
                                                  time.perf_counter() - t0, error=str(e)))
                await d.ack()
                return self._finish(job, JobResult(job_id, outcome, time.perf_counter() - t0,
                                              job.stats.get("uploaded_bytes", 0)))
        except Exception as e:  # infrastructure error outside the stage loop (e.g. S3 down)
            err = str(e)
            child.error("job failed outside stages", err=err)
            await self.telemetry.emit_status(job_id, api.STATUS_ERRORED)
            outcome = await self._retry(d, attempt, err)
            if outcome == "dead":
                await self._sweep_uploads(job, child)
            return self._finish(job, JobResult(job_id, outcome, time.perf_counter() - t0, error=err))
        finally:
            self.active.pop(slot, None)
            self.metrics.inflight.dec()
            await self._release_jobdir(job, job.stats.get("outcome", ""))

    async def _release_jobdir(self, job: Job, outcome: str) -> None:
        """Keep a failed attempt's partial data for the retry (resume); drop it when the job
        is finished for good (dead-lettered, or stalled with cleanup_on_stall, App. A #6)."""
        jd = job.jobdir
        if jd is None:
            return
        drop = outcome == "dead" or (outcome == "stalled" and self.cfg.download.cleanup_on_stall)
        loop = asyncio.get_running_loop()
        if drop or not jd.exclusive:
            reaper = get_reaper(self.services)
            if reaper.background:
                try:
                    reaper.reap(jd.path)
                except ValueError as e:
                    job.logger.error("job dir not removed", err=str(e))
            else:
                await loop.run_in_executor(None, jd.remove)
        jd.release()
        job.jobdir = None

    def _finish(self, job: Optional[Job], r: JobResult) -> JobResult:
        if job is not None:
            job.stats["outcome"] = r.outcome
            r.stats = job.stats
        self.results.append(r)
        self.metrics.jobs.labels(r.outcome).inc()
        self.metrics.job_duration.labels(r.outcome).observe(r.seconds)
        if self.on_result is not None:
            self.on_result(r)
        return r

    async def _sweep_uploads(self, job: Job, log: Logger) -> None:
        """The job is finished for good: abort the multipart uploads still open under its
        originals (a worker killed mid-relay, a resumable upload kept for a retry that then
        went another way, a disk upload kept for resume) and delete its relay journals.
        Best effort - a failure here never changes the job's outcome. The reference leaves
        this to a bucket lifecycle rule (minio-js aborts only its own failed uploads)."""
        if not self.cfg.s3.sweep_stale_uploads:
            return
        b = self.cfg.s3.bucket
        job_id = job.media.id
        try:
            n = 0
            for key, uid in await self.s3.list_uploads(b, keys.originals_prefix(job_id)):
                try:
                    await self.s3.abort_multipart_upload(b, key, uid)
                    n += 1
                except S3Error:
                    pass
            for it in await self.s3.list_objects(b, keys.journal_prefix(job_id)):
                try:
                    await self.s3.delete_object(b, it.name)
                except S3Error:
                    pass
            if n:
                self.metrics.stale_uploads.inc(n)
                job.stats["stale_uploads_aborted"] = n
                log.info("aborted stale multipart uploads", count=n)
        except Exception as e:        # noqa: BLE001 - cleanup must not fail the job
            log.warn("stale upload sweep failed", err=str(e))

    async def _already_staged(self, job_id: str, log: Logger) -> bool:
        log.info("checking s3 bucket to see if files already exist for id", job_id)
        try:
            await self.s3.get_object(self.cfg.s3.bucket, keys.done_key(job_id))
            return True
        except S3Error as e:
            if e.not_found:
                log.info("failed to find done file in staging")
                return False
            raise

    async def _run_stages(self, job: Job, slot: int) -> None:
        last: Any = {}
        for name, fn in self.stages:
            job.logger.info(f"invoking stage '{name}'")
            self.active[slot].stage = name
            job.last_stage = last
            ts = time.perf_counter()
            with self.tracer.span(f"stage.{name}"), self.metrics.time_stage(name):
                last = await fn(job)
            job.stats.setdefault("stage_s", {})[name] = round(time.perf_counter() - ts, 4)
            job.emitter.emit("progress", 0)

    async def _retry(self, d: Delivery, attempt: int, err: str) -> str:
        b = self.cfg.broker
        if self.cfg.mode == "reference":
            await d.nack(requeue=True)
            return "failed"
        if attempt >= b.max_retries:
            await self._dead_letter(d, err)
            return "dead"
        delay = min(b.retry_backoff_max_s, b.retry_backoff_s * (2 ** attempt))
        hdrs = dict(d.headers)
        hdrs["x-attempt"] = attempt + 1
        hdrs["x-last-error"] = redact_text(err)[:512]
        try:
            if b.retry_delay == "queue":
                # the broker holds the message for `delay`; this delivery (and its prefetch
                # slot) is released right away, so healthy jobs never queue behind a backoff
                await self.broker.publish_delayed(b.download_queue, d.body, hdrs, delay)
            else:
                await asyncio.sleep(delay)
                await self.broker.publish(b.download_queue, d.body, hdrs)
        except Exception:
            await d.nack(requeue=True)
            return "failed"
        self.metrics.retries.inc()
        await d.ack()
        return "retried"

    async def _dead_letter(self, d: Delivery, err: str) -> None:
        hdrs = dict(d.headers)
        hdrs["x-last-error"] = redact_text(err)[:512]
        try:
            await self.broker.publish(self.cfg.broker.dead_letter_queue, d.body, hdrs)
            await d.ack()
        except Exception:
            await d.nack(requeue=True)

    # ------------------------------------------------------------------ direct API
    async def submit(self, msg: Any, headers: Optional[Dict[str, Any]] = None) -> None:
        await self.broker.publish(self.cfg.broker.download_queue, api.encode(msg), headers)

    def health(self) -> Tuple[int, Dict[str, Any]]:
        """``GET /health`` body/status (lib/main.js:176-192)."""
        import os as _os
        import socket
        n = len(self.active)
        if n == 0 and self.cfg.health.legacy_idle_500:
            return 500, {"message": "Not Running Jobs"}
        return 200, {"metadata": {"success": True, "host": socket.gethostname(),
                                  "pid": _os.getpid()},
                     "data": {"active": n}}
