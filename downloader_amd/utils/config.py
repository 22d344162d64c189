"""Typed configuration (the reference's ``triton-core/config`` + env flags + constants).

Reference behaviour:
  * ``await Config('converter')`` loads a named YAML config (index.js:18; the name is a
    copy/paste bug, App. A #1).  We load ``downloader`` and accept ``converter`` as an alias.
  * keys used: ``instance.download_path`` (lib/download.js:235,240) and the S3 settings read
    by ``minio.newClient(config)`` (lib/main.js:41).
  * env: ``PORT`` (lib/main.js:194), ``ALLOW_FILE_URLS`` (lib/download.js:178).
  * every hard-coded constant (TIMEOUT=240000 lib/download.js:21, 30 s ticker :88, bucket name
    lib/upload.js:29, media extensions lib/process.js:15-20, prefetch 1 lib/main.js:46)
    becomes a field here with the reference value as default.

Precedence: defaults < YAML file < ``STAGER_<SECTION>__<FIELD>`` env < explicit overrides.
``mode: reference`` pins the reference's throughput-relevant structure (one job in flight,
sequential files, sequential parts, one HTTP stream) for A/B benchmarking.
"""
from __future__ import annotations

import os
from pathlib import Path
from typing import Any, Dict, List, Literal, Mapping, Optional

import yaml
from pydantic import BaseModel, Field

MiB = 1024 * 1024


class InstanceConfig(BaseModel):
    # job dirs live in <download_path>/<media.id>; relative = under the project root
    # (lib/download.js:234-240)
    download_path: str = "downloads"
    # App. A #18: concurrent duplicate deliveries must not share a directory.
    per_attempt_dirs: bool = True
    # Finished job dirs are renamed into <download_path>/.trash and unlinked by a background
    # thread instead of inline before the convert publish (reference: inline rm, upload.js:60).
    background_cleanup: bool = True


class S3Config(BaseModel):
    endpoint: str = "127.0.0.1:9000"            # host:port, or a URL whose scheme sets `secure`
    access_key: str = "minioadmin"
    secret_key: str = "minioadmin"              # masked in `config` output unless --show-secrets
    session_token: str = ""                     # temporary (STS) credentials: x-amz-security-token
    # SigV4 signing region; a bucket elsewhere is learnt from the server's refusal
    region: str = "us-east-1"
    secure: bool = False                        # https to S3 (minio-js useSSL)
    # staging bucket, created if missing (lib/upload.js:29-30)
    bucket: str = "triton-staging"
    # minio-js 7 default; per-request Python cost (SigV4, executor hop) makes fewer, larger
    # parts faster even for the socket relay: 100 MB jobs 37 GB/s @16 MiB -> 47.5 GB/s @64 MiB
    part_size: int = 64 * MiB
    # Objects up to this size go in ONE PUT (socket relay or sendfile), larger ones as
    # multipart uploads of part_size parts - minio-js' split (lib/upload.js:45 fPutObject), so a
    # 100 MB object is 2 parts relayed in parallel. Round 2 used 128 MiB (one PUT per 100 MB
    # job); bench.py reports that setting in the same call as `single_put_MBps`.
    multipart_threshold: int = 64 * MiB
    max_inflight_parts: int = 8                 # multipart parts in flight per object (ref: 1)
    # objects uploaded at once per job (ref: 1, lib/upload.js:34-52)
    concurrent_files: int = 4
    # Sign with UNSIGNED-PAYLOAD (body never re-read for SHA-256); when False the
    # native hasher computes the payload SHA-256 (minio-js over plain HTTP does that).
    unsigned_payload: bool = True
    # Content-Type of staged media from the file extension (minio-js fPutObject looks it up
    # with mime-types: .mkv -> video/x-matroska, ...); False: application/octet-stream.
    content_type_by_extension: bool = True
    # Keep a failed multipart upload open and, on the retry, re-use the parts whose ETag
    # equals the local MD5 of the same range.
    resume_uploads: bool = True
    # Use the native zero-copy HTTP transport for plain-http endpoints.
    native_transport: bool = True
    # auto: virtual-hosted-style (<bucket>.<endpoint>) for AWS endpoints like minio-js,
    # path-style elsewhere (MinIO); or force "path" / "virtual"
    addressing: Literal["auto", "path", "virtual"] = "auto"
    # Over TLS a relay is bound by one thread's AES-GCM: objects > 6 MiB under the multipart
    # threshold are relayed as up to max_inflight_parts parallel parts instead of one PUT
    split_tls_relays: bool = True
    # payload integrity per PUT / part: CRC32C (x-amz-checksum-crc32c) the server verifies.
    # always (default) = every PUT and part, the plain splice relay included (it peeks each
    # byte once into user space for the CRC: +0.08 worker CPU-s/GB); auto = only where bytes
    # cross user space anyway (memory, disk uploads, TLS relays, piece-hashed torrent relays:
    # the plain relay then carries no payload checksum); off. minio-js hashes every byte it
    # uploads: Content-MD5 over https / a signed SHA-256 over http (lib/upload.js:45).
    checksum: Literal["auto", "always", "off"] = "always"
    connect_timeout_s: float = 10.0
    request_timeout_s: float = 300.0            # socket idle timeout of one request
    # retries of a retryable S3 error (5xx, SlowDown, resets) with jittered backoff
    retries: int = 3
    # streamed relays of objects at least this large keep a resume journal (<id>/.stager/):
    # a failed attempt leaves its multipart upload for the job's retry, which relays only the
    # parts not uploaded yet from the same (pinned) source version; 0 = off
    relay_resume_min_bytes: int = 1 << 30
    # when a job ends for good (staged after a retry or a redelivery, or dead-lettered),
    # abort the multipart uploads still open under <id>/original/ and drop its resume
    # journals: what a killed worker or a kept attempt left behind is not billed forever
    sweep_stale_uploads: bool = True


class BrokerConfig(BaseModel):
    # amqp (RabbitMQ or the bundled broker) or memory (tests, benches)
    backend: Literal["amqp", "memory"] = "amqp"
    url: str = ""  # empty -> dynamics('rabbitmq')
    prefetch: int = 1          # lib/main.js:46 (AMQP arg 1)
    max_retries: int = 2       # lib/main.js:46 (AMQP arg 2, INFERRED as retry budget)
    download_queue: str = "v1.download"   # lib/main.js:172
    convert_queue: str = "v1.convert"     # lib/main.js:164
    dead_letter_queue: str = "v1.download.dead" # jobs that used up max_retries are published here
    # first re-publish delay of a failed job (doubles per attempt)
    retry_backoff_s: float = 0.5
    retry_backoff_max_s: float = 30.0
    heartbeat_s: int = 30                       # AMQP heartbeat (0: off)
    # a publish (convert job, retry, dead letter) waits this long for a lost connection to
    # come back before it fails (amqp-connection-manager keeps retrying forever)
    publish_retry_s: float = 120.0
    # first reconnect delay after a lost connection (doubles, max 30 s)
    reconnect_delay_s: float = 1.0
    connect_retry_s: float = 60.0               # keep retrying the first connect this long
    # first wait before reopening a channel the broker closed (consumer_timeout, 406) or
    # re-consuming after a broker basic.cancel (queue deleted); doubles, max 30 s
    recover_delay_s: float = 1.0
    # failed-job backoff: "queue" = ack now and re-publish through a TTL holding queue that
    # dead-letters back to download_queue (no prefetch slot held while waiting); "sleep" =
    # wait inside the consumer, holding the delivery (round-2 behaviour, kept for A/B)
    retry_delay: Literal["queue", "sleep"] = "queue"
    # PEM CA bundle for amqps:// (default: tls.ca_file)
    ca_file: str = ""
    # client certificate (PEM) for amqps:// brokers that require one (mutual TLS); key_file
    # empty: the key is in cert_file
    cert_file: str = ""
    key_file: str = ""


class TelemetryConfig(BaseModel):
    enabled: bool = True                        # status / progress messages (triton-core telemetry)
    status_queue: str = "v1.telemetry.status"
    progress_queue: str = "v1.telemetry.progress"
    # emits never wait for the broker: they go to a bounded outbox that one task flushes in
    # order, each publish bounded by this; a failed one is retried (backoff up to
    # retry_max_s) while newer events queue behind it
    publish_timeout_s: float = 1.0
    retry_max_s: float = 5.0
    buffer_max: int = 10_000                    # outbox bound: past it the oldest is dropped


class DownloadConfig(BaseModel):
    torrent_metadata_timeout_s: float = 240.0   # lib/download.js:21,47-50
    torrent_stall_timeout_s: float = 240.0      # lib/download.js:90-101
    progress_interval_s: float = 30.0           # lib/download.js:88
    allow_file_urls: bool = False               # env ALLOW_FILE_URLS (lib/download.js:178)
    http_streams: int = 4                       # parallel Range GETs per file (ref: 1)
    # smallest Range slice when a file is split over http_streams
    http_min_split: int = 32 * MiB
    http_timeout_s: float = 300.0
    http_min_rate: float = 0.0                  # bytes/s stall floor, 0 = off
    http_native: bool = True                    # native splice() transport for http://
    # Forward proxy for http(s) SOURCE fetches, as request@2 does: "env" = HTTP_PROXY /
    # HTTPS_PROXY / NO_PROXY, "" = never, or http://[user:pass@]host:port (net/proxy.py).
    http_proxy: str = "env"
    # Single selector-approved HTTP file -> relayed origin->S3 socket-to-socket (no disk hop).
    stream_http: bool = True
    # Torrents: stage selected files part by part while the torrent is still downloading.
    eager_upload: bool = True
    # Webseed-only .torrent jobs: relay each S3 part webseed->S3 with in-flight SHA-1 and no
    # disk hop (torrent/stream.py). auto: when the metainfo lists no trackers, first attempt
    # only (a retry takes the disk path with every source); always: whenever webseeds exist.
    torrent_stream: Literal["auto", "always", "off"] = "auto"
    # parts (Range GETs) in flight per job: config 4, pinned A/B, 16 / 24 / 32: gfx950 arm
    # 30.9 - 31.3 / 31.9 / 33.2 GB/s, host arm 26.1 - 26.6 / 27.9 / 27.8 (each relay leaves
    # its thread ~half idle waiting on the webseed; profiles/r6/split/stream_parallel/)
    torrent_stream_parallel: int = 32
    # Byte budget of the streamed relay's part buffers (one per part in flight, as large as
    # the part): relays in flight, parts awaiting their DMA to the GPU and idle pooled buffers
    # of ALL jobs of the worker draw from it, so their resident memory never exceeds it
    # (utils/membudget.py). 0 = relay_memory_fraction of this worker's share of the memory
    # limit (cgroup memory.max, else RAM, / worker processes in the container).
    relay_memory_mb: int = 0
    relay_memory_fraction: float = 0.25
    # idle seconds after the last stream-staged job before the hashed relay's pooled part
    # buffers are unmapped; jobs inside the window reuse them without re-faulting ~1 GiB of
    # huge pages (MI355X box, 4 GB torrent: 26.7 - 27.8 GB/s warm vs 19.2 - 20.0 GB/s when
    # every job faults its buffers afresh). Idle buffers always stay inside the budget above.
    relay_pool_idle_trim_s: float = 60.0
    # Splice pipe capacity per transfer in KiB (relays, HTTP bodies to disk). 0: derived from
    # the user's pipe page budget (fs.pipe-user-pages-soft, 64 MiB by default for non-root
    # users, shared by every process of that uid - containers of one uid on a host included)
    # split over `pipe_sharers` processes of ~16 transfers each; 1 MiB when unbounded (root).
    # Past the budget pipes shrink to two pages, so transfers copy through user space instead.
    pipe_kb: int = 0
    pipe_sharers: int = 4
    bucket_concurrency: int = 4                 # ref: sequential fGetObject (lib/download.js:218)
    bucket_secure: bool = True                  # bucket:// is always TLS in the reference
    # bucket:// sources: select media from the object listing and relay only the selected
    # objects source S3 -> staging S3 through presigned GETs (no disk hop, extras never fetched)
    stream_bucket: bool = True
    # ... and when the source bucket lives on the staging endpoint with the same credentials,
    # copy server-side (CopyObject / UploadPartCopy): no bytes through the worker
    bucket_server_copy: bool = True
    # file:// sources: a single selector-approved file is uploaded straight from its path
    # (sendfile) instead of being copied into the job directory first
    stream_file: bool = True
    # torrent piece SHA-1: cpu, gpu (gfx950 kernel) or auto
    verify_backend: Literal["cpu", "gpu", "auto"] = "auto"
    # streamed torrents (torrent_stream): pieces of each relayed part hashed by the host
    # multi-buffer SHA-1 (cpu) or by the gfx950 PartHasher (gpu: batched one-lane-per-piece
    # launches; the relay slot is freed when the part's bytes are moved, digests arrive in a
    # continuation)
    # auto: the GPU for jobs with more parts than stream_gpu_tail, when stream jobs share the
    # worker, or when the host lacks AVX-512 (set up on an executor thread the first time it
    # is wanted; profiles/archive/r3_relayhash4/, r3_tail2/)
    stream_verify_backend: Literal["cpu", "gpu", "auto"] = "auto"
    # parts awaiting GPU digests across all jobs of the worker: ~128 - 160 hide the device's
    # per-piece latency (profiles/archive/r3_relayhash*/). A part holds its host buffer (and budget)
    # only until its DMA into an HBM slot is over.
    stream_gpu_pending: int = 160
    # PartHasher device slots (1 GiB of HBM each): enough that a part's DMA never waits for a
    # kernel to free a slot, which is what keeps the host buffers short-lived
    stream_gpu_slots: int = 16
    # bytes per slot (MiB): one sha1_lanes launch hashes up to slot / piece_len pieces, so
    # with 4 MiB pieces a 1 GiB slot caps a launch at 256 lanes (~15 GB/s per busy stream)
    stream_gpu_slot_mb: int = 1024
    # PartHasher streams: copy streams for the parts' DMAs, compute streams for the kernels
    # (0 = the hardware queues the copy streams leave, GPU_MAX_HW_QUEUES = 4 by default): a
    # copy stream sharing a hardware queue with a compute stream waits behind its kernels.
    # Config 4 at a 1 GiB part budget, 6 steady reps each: 2 copy + 2 compute 29.3 GB/s
    # median, 1 + 3 27.1, round 3's 1 + 4 25.8 (profiles/archive/r4/copies/)
    stream_gpu_copy_streams: int = 2
    stream_gpu_compute_streams: int = 0
    stream_gpu_min_pieces: int = 8              # parts with fewer whole pieces stay on the host
    # once fewer parts than this are queued, the job's remaining parts hash on the host (the
    # GPU's per-piece latency would otherwise land on the end of the job). With sha1_lanes
    # (73 - 100 ms a launch) 16 / 48 / 96 / 128 / 160 gave 21.2 - 21.8 / 22.7 - 23.6 / 25.0 -
    # 29.1 / 25.7 - 28.5 / 24.4 - 27.5 GB/s for one 20 GB job vs 22.7 - 25.4 on the host
    # (profiles/archive/r3_tail*/); with sha1_lanes_split (57 ms), pinned like bench.py's rank:
    # 32 parts 34.0 vs 28.0 GB/s (1.22x, 85 % of the parts on the device), 16 parts 30.7 vs
    # 26.2 (1.17x, 90 %); 1 copy + 3 compute streams 1.16 - 1.17x (profiles/r6/split/
    # stream_tail/call3_pinned/; the unpinned calls beside it show both arms throttled alike)
    stream_gpu_tail: int = 32
    verify_threads: int = 0                     # host SHA-1 threads per check (0: usable CPUs)
    # Initialise the GPU verifier at worker start (device = worker index % GPUs; a no-op
    # without a HIP device) so "auto" sends rechecks >= 256 MiB and the webseed runs of
    # torrents >= 8 GiB to the GPU instead of paying the cold start inside a job.
    gpu_prewarm: bool = True
    torrent_listen_port: int = 0                # incoming peer connections (0: any free port)
    torrent_max_peers: int = 32
    torrent_enable_dht: bool = True             # BEP-5 mainline DHT
    # DHT bootstrap nodes ("host:port"); empty = the public mainline routers
    torrent_dht_bootstrap: List[str] = Field(default_factory=list)
    # trackers announced to for a bare-infohash torrent id (it carries none itself;
    # webtorrent's `announce` option) - the DHT finds peers either way
    torrent_default_trackers: List[str] = Field(default_factory=list)
    torrent_enable_trackers: bool = True        # HTTP / UDP trackers
    torrent_enable_webseeds: bool = True        # BEP-19 url-list
    torrent_request_pipeline: int = 16          # 16 KiB block requests in flight per peer
    # peer connections framed, assembled, SHA-1'd (16 pieces at a time) and written by the
    # native wire after the handshake (csrc/peerwire.cpp); False: all in Python (peer.py)
    torrent_native_wire: bool = True
    # the native wire requests whole pieces assigned to a connection by itself, keeping the
    # pipeline full from its reader thread (Python books a piece, not 256 blocks); the endgame
    # and pieces a choking / closing peer leaves go back to per-block requests
    torrent_wire_requests: bool = True
    # SHA-1 of swarm pieces on the native wire: "cpu" = the host multi-buffer SHA-1 (16 pieces
    # at a time), "gpu" = the gfx950 PartHasher (set up once per worker), "auto" = the device
    # for torrents of swarm_gpu_min_gb and up (0: never) or on hosts without the AVX-512
    # multi-buffer SHA-1, else the host. Round 5 kept the device for 8 GB and up (2 GB: 5.3 -
    # 5.8 vs 8.9 - 9.2 GB/s on the host - the last pieces' device latency on the job's end);
    # with the split-wave kernel (57 vs 73 ms per 4 MiB piece) and the auto host tail below,
    # config 6 runs within ~5 % of the host at 2 GB and 16 GB on less CPU (profiles/r6/tail/)
    swarm_verify_backend: str = "auto"
    swarm_gpu_min_gb: float = 1.5               # GiB: a "2 GB" (2e9-byte) torrent included
    # native wire threads verifying and writing complete pieces (and, in GPU mode, collecting
    # digests): 2 capped config 6 near 5 - 7 GB/s with pieces queueing behind them
    swarm_verify_threads: int = 4
    # epoll threads reading and writing a session's peer connections on the native wire
    # (connections spread over them): not two threads per connection
    swarm_wire_io_threads: int = 4
    # idle swarm piece buffers kept per worker process (reused: no page faults per piece, and
    # page-locked once in GPU mode, where the download runs up to ~0.5 s ahead of the device).
    # 0: 1/8 of this worker's share of the memory limit, at most 4096 (utils/membudget.py)
    swarm_pool_mb: int = 0
    # GPU mode: pieces on the device at once (a 4 MiB piece spends ~75 ms there plus its wait
    # for a compute stream); past it the host hashes the overflow. 512 overflowed on config 6
    # at 8 GB (6.1 - 6.5 GB/s vs 7.2 - 8.4 with 4096, profiles/archive/r5/swarm/event_loop/)
    swarm_gpu_inflight: int = 1024
    # GPU mode: once no more than this much of the torrent is left to start, pieces are
    # hashed on the host - on the device the last ones would each add their submission ->
    # digest time (~60 - 120 ms) to the end of the job. -1 (auto): the download rate so far x
    # that time as measured (swarm_gpu_tail_x), at most swarm_gpu_tail_max of the torrent; 0:
    # off; > 0: fixed (at most a quarter of the torrent)
    swarm_gpu_tail_mb: int = -1
    # config 6 at 2 GB, steady reps, same calls (profiles/r6/tail/): x 1.3 / at most half
    # 7.4 - 7.9 GB/s vs host 8.3 - 9.2; x 2 / 3/4 7.4 - 8.0 vs 8.1 - 9.2; x 3 / 0.85 7.9 - 8.4
    # vs 8.1 - 9.2 (the device takes the first ~20 % of such a torrent: what it can hand back
    # before the download ends)
    swarm_gpu_tail_x: float = 3.0               # auto tail: x the measured device latency
    swarm_gpu_tail_max: float = 0.85            # auto tail: at most this share of the torrent
    # complete swarm pieces waiting for their SHA-1 (host verifiers, the device) or the writer
    # hold their buffers; at this much no new piece is started until half has drained. Without
    # it a download faster than its verification ran GBs ahead (config 6 at 16 GB: 4 - 8 GB).
    # 0: like swarm_pool_mb
    swarm_backlog_mb: int = 0
    webseed_streams: int = 4                    # concurrent Range GETs per webseed (0: http_streams)
    webseed_chunk: int = 64 * MiB               # bytes of whole pieces per webseed request run
    webseed_verify_depth: int = 2               # fetched runs hashing while a stream fetches on
    webseed_verify_depth_gpu: int = 32          # same when runs are verified by the GPU batcher
    # Disk paths (HTTP to disk, torrents to disk) check before writing that the staging
    # filesystem holds what is still to be written plus this reserve (stages/space.py)
    min_free_bytes: int = 0
    cleanup_on_stall: bool = True               # App. A #6 (reference leaves data behind)
    emit_errored_on_stall: bool = False         # App. A #6 (reference: ack silently)


class ProcessConfig(BaseModel):
    # kept extensions (lib/process.js:15-20)
    media_exts: List[str] = Field(default_factory=lambda: [".mp4", ".mkv", ".mov", ".webm"])
    case_insensitive_exts: bool = False         # App. A #15 (reference: case-sensitive)
    legacy_full_path_extras: bool = False       # App. A #14
    legacy_any_depth_sole_dir: bool = False     # App. A #16


class HealthConfig(BaseModel):
    # GET /health (+ /healthz, /readyz, /metrics) on port
    enabled: bool = True
    host: str = "0.0.0.0"
    port: int = 3401                            # lib/main.js:194 (env PORT)
    legacy_idle_500: bool = True                # App. A #9


class MetricsConfig(BaseModel):
    enabled: bool = True                        # Prometheus metrics (triton-core prom)
    # /metrics is served on the health port; a dedicated port may be set as well.
    port: int = 0


class TraceConfig(BaseModel):
    # per-job / per-stage spans, traceparent in message headers
    enabled: bool = False
    path: str = ""                              # JSONL span sink ("" -> stderr when enabled)


class TlsConfig(BaseModel):
    """TLS for https:// sources, S3 with ``secure: true`` and bucket:// (always TLS)."""
    verify: bool = True                         # False: accept any certificate
    ca_file: str = ""                           # extra PEM trust (private CA), beside the system store
    # TLS in the native transport (OpenSSL on the transfer threads, csrc/tls.cpp); False
    # sends https through aiohttp on the event loop (one core per process for all streams)
    native: bool = True


class Config(BaseModel):
    # config name (the reference loads `converter`, App. A #1; both names are searched)
    name: str = "downloader"
    # tuned, or reference = the reference's serial structure (BASELINE.md comparison mode)
    mode: Literal["tuned", "reference"] = "tuned"
    concurrency: int = 4                        # jobs in flight per worker process
    instance: InstanceConfig = Field(default_factory=InstanceConfig)
    s3: S3Config = Field(default_factory=S3Config)
    broker: BrokerConfig = Field(default_factory=BrokerConfig)
    telemetry: TelemetryConfig = Field(default_factory=TelemetryConfig)
    download: DownloadConfig = Field(default_factory=DownloadConfig)
    process: ProcessConfig = Field(default_factory=ProcessConfig)
    health: HealthConfig = Field(default_factory=HealthConfig)
    metrics: MetricsConfig = Field(default_factory=MetricsConfig)
    trace: TraceConfig = Field(default_factory=TraceConfig)
    tls: TlsConfig = Field(default_factory=TlsConfig)
    # stage modules in order (`module:factory` plugins allowed, lib/main.js:28-32)
    stages: List[str] = Field(default_factory=lambda: ["download", "process", "upload"])

    def apply_mode(self) -> "Config":
        """``mode: reference`` reproduces the reference's serial structure."""
        if self.mode == "reference":
            self.concurrency = 1
            self.broker.prefetch = 1
            self.s3.concurrent_files = 1
            self.s3.max_inflight_parts = 1
            self.s3.part_size = 64 * MiB             # minio-js 7: 64 MiB parts above 64 MiB
            self.s3.multipart_threshold = 64 * MiB
            # minio-js over plain HTTP signs every PUT/part with its payload SHA-256
            # (SURVEY §2.5); over TLS it would send UNSIGNED-PAYLOAD + Content-MD5 instead.
            self.s3.unsigned_payload = self.s3.secure
            self.s3.checksum = "off"                 # (SHA-256 payload signing checks bytes)
            self.download.http_streams = 1
            self.download.bucket_concurrency = 1
            self.download.webseed_streams = 1
            self.download.webseed_verify_depth = 1   # fetch -> verify -> fetch, one thread
            self.download.verify_backend = "cpu"     # webtorrent hashes on the host,
            self.download.verify_threads = 1         # on its one JS thread (simple-sha1)
            self.download.gpu_prewarm = False
            self.download.stream_http = False
            self.download.eager_upload = False
            self.download.torrent_stream = "off"
            self.instance.background_cleanup = False
        else:
            self.broker.prefetch = max(self.broker.prefetch, self.concurrency)
        return self

    def resolved_download_root(self, repo_root: Optional[Path] = None) -> Path:
        """Relative ``download_path`` resolves against the project root (lib/download.js:234-240)."""
        p = Path(self.instance.download_path)
        if p.is_absolute():
            return p
        root = repo_root or Path(__file__).resolve().parents[2]
        return root / p


def _deep_merge(dst: Dict[str, Any], src: Mapping[str, Any]) -> Dict[str, Any]:
    for k, v in src.items():
        if isinstance(v, Mapping) and isinstance(dst.get(k), dict):
            _deep_merge(dst[k], v)
        else:
            dst[k] = v
    return dst


def _parse_env_value(v: str) -> Any:
    try:
        return yaml.safe_load(v)
    except yaml.YAMLError:
        return v


def env_overrides(env: Mapping[str, str]) -> Dict[str, Any]:
    out: Dict[str, Any] = {}
    for k, v in env.items():
        if not k.startswith("STAGER_"):
            continue
        path = k[len("STAGER_"):].lower().split("__")
        cur = out
        for seg in path[:-1]:
            cur = cur.setdefault(seg, {})
        cur[path[-1]] = _parse_env_value(v)
    # Reference env flags.
    if "PORT" in env:
        out.setdefault("health", {})["port"] = int(env["PORT"])
    if "ALLOW_FILE_URLS" in env:
        out.setdefault("download", {})["allow_file_urls"] = env["ALLOW_FILE_URLS"] == "true"
    return out


def find_config_file(name: str, search: Optional[List[Path]] = None) -> Optional[Path]:
    dirs = search or [Path(os.environ.get("STAGER_CONFIG_DIR", "config")),
                      Path(__file__).resolve().parents[2] / "config"]
    for d in dirs:
        for n in (name, "converter") if name == "downloader" else (name,):
            for ext in (".yaml", ".yml"):
                p = d / f"{n}{ext}"
                if p.is_file():
                    return p
    return None


def load_config(name: str = "downloader", path: Optional[str] = None,
                env: Optional[Mapping[str, str]] = None,
                overrides: Optional[Mapping[str, Any]] = None) -> Config:
    env = os.environ if env is None else env
    data: Dict[str, Any] = {}
    fpath = Path(path) if path else find_config_file(name)
    if fpath is not None:
        with open(fpath, "r", encoding="utf-8") as f:
            loaded = yaml.safe_load(f) or {}
        if not isinstance(loaded, dict):
            raise ValueError(f"config {fpath} must be a mapping")
        _deep_merge(data, loaded)
    _deep_merge(data, env_overrides(env))
    if overrides:
        _deep_merge(data, overrides)
    data.setdefault("name", name)
    return Config.model_validate(data).apply_mode()
