"""Async S3 client (replaces minio-js as wrapped by ``triton-core/minio``).

Operations the reference uses: ``getObject`` (done-marker probe,
lib/main.js:120), ``bucketExists``/``makeBucket`` (lib/upload.js:29-31), ``fPutObject``
(lib/upload.js:45), ``putObject`` with a string body (lib/upload.js:55), ``fGetObject`` and the
``getObjects`` recursive listing (lib/download.js:217-225).

Differences by design:
  * multipart parts are uploaded concurrently (bounded by ``max_inflight_parts``) straight
    from the page cache with ``sendfile``; the reference streams one part at a time.
  * ``fget_object`` can split an object into parallel Range GETs.
  * transient failures (connection errors, 5xx, SlowDown) are retried with backoff.
  * an interrupted multipart upload can be resumed: parts whose ETag equals the local MD5
    of the same range are skipped.
  * payload integrity per PUT / part with S3 flexible checksums (CRC32C) instead of minio-js'
    Content-MD5 / signed SHA-256: ``x-amz-checksum-crc32c`` as a header for
    in-memory and on-disk bodies, as the trailer of an aws-chunked body for socket relays
    (computed while the bytes pass). The server recomputes it and refuses a mismatch with
    400 BadDigest, which is retried. ``checksum``: ``auto`` = wherever the bytes cross user
    space anyway (memory, disk, TLS relays, piece-hashed torrent relays), not the plain
    splice relay; ``always`` = that too (relays then copy through user space); ``off``.
"""
from __future__ import annotations

import asyncio
import json
import os
import random
import re
import xml.etree.ElementTree as ET
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Sequence, Tuple
from urllib.parse import quote

from ..net.http import (FileRange, FileSink, Progress, Response, SourceChanged,
                        TransportError, TransportSet, make_transports, pin_headers)
from ..utils.aio import drain, gather_strict
from ..utils.log import redact_url
from . import sigv4

NS = "{http://s3.amazonaws.com/doc/2006-03-01/}"
COPY_MAX = 5 << 30            # CopyObject limit; larger objects copy as parts
COPY_PART = 512 << 20         # UploadPartCopy range size (server-side: no memory cost here)
_DNS_BUCKET = re.compile(r"^[a-z0-9][a-z0-9.-]{1,61}[a-z0-9]$")
MiB = 1 << 20
MAX_PARTS = 10000
MIN_PART = 5 * MiB


class S3Error(Exception):
    def __init__(self, code: str, message: str = "", status: int = 0, key: str = "",
                 bucket: str = ""):
        super().__init__(f"{code}: {message}" if message else code)
        self.code = code
        self.message = message
        self.status = status
        self.key = key
        self.bucket = bucket

    @property
    def not_found(self) -> bool:
        return self.code in ("NoSuchKey", "NoSuchBucket", "NotFound") or self.status == 404

    @property
    def retryable(self) -> bool:
        # BadDigest / checksum mismatch: bytes corrupted on the way; sending them again (from
        # the file, or a fresh source range) is the remedy
        return self.status >= 500 or self.code in ("SlowDown", "RequestTimeout",
                                                   "InternalError", "ServiceUnavailable",
                                                   "BadDigest", "XAmzContentChecksumMismatch")


@dataclass
class ObjectInfo:
    name: str
    size: int
    etag: str = ""
    last_modified: str = ""
    meta: Dict[str, str] = field(default_factory=dict)   # x-amz-meta-<k> -> value (HEAD)


def _strip(tag: str) -> str:
    return tag.split("}", 1)[-1]


def _find(el: ET.Element, name: str) -> Optional[ET.Element]:
    for c in el:
        if _strip(c.tag) == name:
            return c
    return None


def _text(el: ET.Element, name: str, default: str = "") -> str:
    c = _find(el, name)
    return c.text or default if c is not None else default


def parse_error(resp: Response, bucket: str = "", key: str = "") -> S3Error:
    code, msg = "", ""
    if resp.body:
        try:
            root = ET.fromstring(resp.body)
            code = _text(root, "Code")
            msg = _text(root, "Message")
        except ET.ParseError:
            msg = resp.body[:200].decode("utf-8", "replace")
    if not code:
        code = {404: "NotFound", 403: "AccessDenied", 503: "SlowDown", 500: "InternalError",
                409: "Conflict", 400: "BadRequest"}.get(resp.status, f"HTTP{resp.status}")
        if resp.status == 404 and key:
            code = "NoSuchKey"
    return S3Error(code, msg, resp.status, key, bucket)


class S3Client:
    def __init__(self, endpoint: str, access_key: str, secret_key: str, region: str = "us-east-1",
                 secure: bool = False, transports: Optional[TransportSet] = None,
                 part_size: int = 16 * MiB, multipart_threshold: int = 64 * MiB,
                 max_inflight_parts: int = 8, unsigned_payload: bool = True, retries: int = 3,
                 native: bool = True, connect_timeout: float = 10.0,
                 request_timeout: float = 300.0, ssl_verify: bool = True, ca_file: str = "",
                 native_tls: bool = True, addressing: str = "auto", session_token: str = "",
                 split_tls_relays: bool = True, checksum: str = "auto"):
        if "://" in endpoint:
            secure = endpoint.startswith("https://")
            endpoint = endpoint.split("://", 1)[1]
        self.endpoint = endpoint.rstrip("/")
        self.scheme = "https" if secure else "http"
        self.base = self.scheme + "://" + self.endpoint
        if addressing not in ("auto", "path", "virtual"):
            raise ValueError(f"s3 addressing {addressing!r}: auto, path or virtual")
        self.addressing = addressing
        self.access_key = access_key
        self.secret_key = secret_key
        self.session_token = session_token
        self.split_tls_relays = split_tls_relays
        if checksum not in ("auto", "always", "off"):
            raise ValueError(f"s3 checksum {checksum!r}: auto, always or off")
        self.checksum = checksum
        self.region = region
        # bucket -> region learnt from the server (x-amz-bucket-region / <Region>): an AWS
        # bucket outside the configured region is signed for its own region after the first
        # refusal, as minio-js does with its bucket-location cache
        self._regions: Dict[str, str] = {}
        self._own_transports = transports is None
        self.t = transports or make_transports(native=native, connect_timeout=connect_timeout,
                                               io_timeout=request_timeout,
                                               ssl_verify=ssl_verify, ca_file=ca_file,
                                               native_tls=native_tls)
        self.part_size = max(MIN_PART, part_size)
        self.multipart_threshold = multipart_threshold
        self.max_inflight_parts = max(1, max_inflight_parts)
        self.unsigned_payload = unsigned_payload
        self.retries = retries
        self.resumed_parts = 0      # relayed parts a later attempt found already uploaded

    @classmethod
    def from_config(cls, s3cfg, transports: Optional[TransportSet] = None) -> "S3Client":
        """``minio.newClient(config)`` equivalent (lib/main.js:41, lib/upload.js:20)."""
        return cls(s3cfg.endpoint, s3cfg.access_key, s3cfg.secret_key, s3cfg.region,
                   s3cfg.secure, transports, s3cfg.part_size, s3cfg.multipart_threshold,
                   s3cfg.max_inflight_parts, s3cfg.unsigned_payload, s3cfg.retries,
                   s3cfg.native_transport, s3cfg.connect_timeout_s, s3cfg.request_timeout_s,
                   addressing=s3cfg.addressing, session_token=s3cfg.session_token,
                   split_tls_relays=s3cfg.split_tls_relays, checksum=s3cfg.checksum)

    def virtual_host(self, bucket: str) -> bool:
        """Virtual-hosted-style addressing (``<bucket>.<endpoint>/<key>``) for this bucket?
        ``auto`` follows minio-js 7: AWS endpoints (``*.amazonaws.com``) with a DNS-compatible
        bucket name, except names with dots over https (they break the wildcard certificate);
        everything else (MinIO, the fakes) path-style."""
        if not bucket or self.addressing == "path":
            return False
        if self.addressing == "virtual":
            return True
        host = self.endpoint.rsplit(":", 1)[0].lower()
        if not (host == "amazonaws.com" or host.endswith(".amazonaws.com")):
            return False
        if not _DNS_BUCKET.match(bucket) or ".." in bucket:
            return False
        return "." not in bucket or self.scheme == "http"

    def presign(self, method: str, bucket: str, key: str, expires: int = 3600) -> str:
        """Presigned URL (query-string SigV4, minio-js ``presignedUrl``): any HTTP client -
        the socket relay included - can then GET the object, Range requests too."""
        host, path = self._address(bucket, key)
        q = sigv4.presign(method, host, path, [], self.access_key, self.secret_key,
                          self.region_of(bucket), expires, session_token=self.session_token)
        return f"{self.scheme}://{host}" + sigv4.uri_encode(path, True) + "?" + \
            sigv4.canonical_query(q)

    def region_of(self, bucket: str) -> str:
        return self._regions.get(bucket, self.region)

    def _region_hint(self, resp: Response, bucket: str) -> Optional[str]:
        """The bucket's real region when the server refused the signing region, else None."""
        if not bucket or resp.status not in (301, 400, 403):
            return None
        r = resp.header("x-amz-bucket-region") or ""
        if not r and resp.body:
            try:
                r = _text(ET.fromstring(resp.body), "Region")
            except ET.ParseError:
                r = ""
        return r if r and r != self.region_of(bucket) else None

    def _address(self, bucket: str, key: str) -> Tuple[str, str]:
        """(Host header, canonical URI path) of an object or bucket request."""
        if self.virtual_host(bucket):
            return f"{bucket}.{self.endpoint}", "/" + key
        return self.endpoint, "/" + bucket + ("/" + key if key else "")

    async def close(self) -> None:
        if self._own_transports:
            await self.t.close()

    # ------------------------------------------------------------------ request core
    async def _payload_hash(self, body) -> str:
        if body is None:
            return sigv4.EMPTY_SHA256
        if self.unsigned_payload:
            return sigv4.UNSIGNED
        from ..ops import native
        if isinstance(body, FileRange):
            h = native().Hasher("sha256")
            await asyncio.get_running_loop().run_in_executor(
                None, h.update_fd, body.fd, body.offset, body.length)
            return h.hexdigest()
        return native().digest("sha256", body).hex()

    def want_checksum(self, relay: bool = False, tls: bool = False, hashed: bool = False) -> bool:
        """Send a CRC32C with this upload? (``checksum`` policy, see the module docstring)."""
        if self.checksum == "off":
            return False
        if self.checksum == "always" or not relay:
            return True
        return tls or hashed

    async def _checksum_header(self, body) -> str:
        from ..ops import hashing
        if isinstance(body, FileRange):
            return await asyncio.get_running_loop().run_in_executor(
                None, hashing.crc32c_fd_b64, body.fd, body.offset, body.length)
        return hashing.crc32c_b64(body)

    async def _request(self, method: str, bucket: str, key: str = "",
                       query: Sequence[Tuple[str, str]] = (), body=None,
                       headers: Optional[Dict[str, str]] = None, sink: Optional[FileSink] = None,
                       progress: Optional[Progress] = None, ok: Sequence[int] = (),
                       expect_body: bool = True, checksum: bool = False) -> Response:
        host, path = self._address(bucket, key)
        qs = sigv4.canonical_query(query)
        url = f"{self.scheme}://{host}" + sigv4.uri_encode(path, True) + ("?" + qs if qs else "")
        phash = await self._payload_hash(body)
        if checksum and body is not None:
            headers = dict(headers or {})
            headers["x-amz-checksum-crc32c"] = await self._checksum_header(body)
        attempt = 0
        relocated = False
        while True:
            hdrs = {"host": host}
            if self.session_token:
                hdrs["x-amz-security-token"] = self.session_token
            if headers:
                hdrs.update({k.lower(): v for k, v in headers.items()})
            sigv4.sign(method, path, list(query), hdrs, self.access_key, self.secret_key,
                       self.region_of(bucket), phash)
            try:
                if sink is not None and attempt > 0:
                    sink.max_bytes = sink.max_bytes  # body rewritten from the same offset
                resp = await self.t.request(method, url, headers=list(hdrs.items()), body=body,
                                            sink=sink, progress=progress,
                                            expect_body=expect_body)
            except TransportError as e:
                err: Exception = e
                retry = True
            else:
                if 200 <= resp.status < 300 or resp.status in ok:
                    resp.sent_checksum = (headers or {}).get("x-amz-checksum-crc32c", "")
                    return resp
                hint = None if relocated else self._region_hint(resp, bucket)
                if hint:                # re-sign for the bucket's region, at once
                    self._regions[bucket] = hint
                    relocated = True
                    continue
                err = parse_error(resp, bucket, key)
                retry = err.retryable
            if not retry or attempt >= self.retries:
                raise err
            attempt += 1
            await asyncio.sleep(min(5.0, 0.1 * (2 ** attempt)) * (0.5 + random.random()))

    # ------------------------------------------------------------------ buckets
    async def bucket_exists(self, bucket: str) -> bool:
        r = await self._request("HEAD", bucket, ok=(404,), expect_body=False)
        return r.status != 404

    async def make_bucket(self, bucket: str) -> None:
        body = b""
        if self.region and self.region != "us-east-1":
            body = (f'<CreateBucketConfiguration xmlns="{NS[1:-1]}"><LocationConstraint>'
                    f"{self.region}</LocationConstraint></CreateBucketConfiguration>").encode()
        try:
            await self._request("PUT", bucket, body=body)
        except S3Error as e:
            if e.code not in ("BucketAlreadyOwnedByYou", "BucketAlreadyExists"):
                raise

    async def ensure_bucket(self, bucket: str) -> None:
        if not await self.bucket_exists(bucket):
            await self.make_bucket(bucket)

    # ------------------------------------------------------------------ objects
    async def get_object(self, bucket: str, key: str) -> bytes:
        r = await self._request("GET", bucket, key)
        return r.body

    async def head_object(self, bucket: str, key: str) -> ObjectInfo:
        r = await self._request("HEAD", bucket, key, ok=(404,), expect_body=False)
        if r.status == 404:
            raise S3Error("NoSuchKey", "", 404, key, bucket)
        return ObjectInfo(key, int(r.header("content-length", "0") or 0),
                          (r.header("etag") or "").strip('"'), r.header("last-modified") or "",
                          {k[11:]: v for k, v in r.headers if k.startswith("x-amz-meta-")})

    async def object_exists(self, bucket: str, key: str) -> bool:
        try:
            await self.head_object(bucket, key)
            return True
        except S3Error as e:
            if e.not_found:
                return False
            raise

    async def put_object(self, bucket: str, key: str, data, content_type: str = "") -> str:
        if isinstance(data, str):
            data = data.encode("utf-8")
        hdrs = {"content-type": content_type} if content_type else None
        r = await self._request("PUT", bucket, key, body=bytes(data), headers=hdrs,
                                checksum=self.want_checksum())
        return (r.header("etag") or "").strip('"')

    async def delete_object(self, bucket: str, key: str) -> None:
        await self._request("DELETE", bucket, key, ok=(404,))

    async def fput_object(self, bucket: str, key: str, path: str,
                          progress: Optional[Progress] = None, resume: bool = False,
                          concurrency: Optional[int] = None, content_type: str = "") -> str:
        """minio-js ``fPutObject``: one PUT up to the multipart threshold, else a multipart
        upload; ``content_type`` goes on the PUT / the multipart initiation."""
        size = os.path.getsize(path)
        fd = os.open(path, os.O_RDONLY | getattr(os, "O_CLOEXEC", 0))
        hdrs = {"content-type": content_type} if content_type else None
        try:
            if size <= self.multipart_threshold:
                r = await self._request("PUT", bucket, key, body=FileRange(fd, 0, size),
                                        progress=progress, headers=hdrs,
                                        checksum=self.want_checksum())
                return (r.header("etag") or "").strip('"')
            return await self._multipart(bucket, key, fd, size, path, progress, resume,
                                         concurrency or self.max_inflight_parts, content_type)
        finally:
            os.close(fd)

    def plan_parts(self, size: int, align_offset: int = 0, align: int = 0,
                   part_size: int = 0) -> List[Tuple[int, int, int]]:
        """(part number, offset, length) of a multipart upload of ``size`` bytes.

        ``align``/``align_offset``: the object is bytes [align_offset, align_offset + size) of
        a larger stream cut into ``align``-sized units (torrent pieces). When the part size is
        a multiple of ``align``, the first part is shortened so every interior part boundary
        falls on a unit boundary: a torrent piece then never straddles two parts, so only
        pieces at the file's two ends need assembling from fragments. S3 allows unequal
        parts (all but the last >= 5 MiB). ``part_size``: instead of ``self.part_size``."""
        ps = max(MIN_PART, part_size) if part_size else self.part_size
        while (size + ps - 1) // ps > MAX_PARTS:
            ps *= 2
        first = ps
        if align > 0 and ps % align == 0 and size > ps:
            first = ps - align_offset % align
            while first < MIN_PART:            # part size close to the 5 MiB floor
                first += align
        out, off, num = [], 0, 1
        while off < size:
            ln = min(first if num == 1 else ps, size - off)
            out.append((num, off, ln))
            off += ln
            num += 1
        if len(out) > MAX_PARTS:               # the shortened first part added one: fall back
            return [(i + 1, o, min(ps, size - o)) for i, o in enumerate(range(0, size, ps))]
        return out

    async def _multipart(self, bucket: str, key: str, fd: int, size: int, path: str,
                         progress: Optional[Progress], resume: bool, concurrency: int,
                         content_type: str = "") -> str:
        parts = self.plan_parts(size)
        upload_id = None
        done: Dict[int, str] = {}
        if resume:
            upload_id = await self.find_upload(bucket, key)
            if upload_id:
                done = await self._reusable_parts(bucket, key, upload_id, path, parts)
        if not upload_id:
            upload_id = await self.create_multipart_upload(bucket, key, content_type,
                                                           checksum=self.want_checksum())
        sem = asyncio.Semaphore(concurrency)
        etags: Dict[int, str] = dict(done)

        async def one(num: int, off: int, ln: int) -> None:
            async with sem:
                etags[num] = await self.upload_part(bucket, key, upload_id, num,
                                                    FileRange(fd, off, ln), progress)

        try:
            await gather_strict(*(one(n, o, ln) for n, o, ln in parts if n not in done))
            return await self.complete_multipart_upload(
                bucket, key, upload_id, [(n, etags[n]) for n, _, _ in parts])
        except BaseException:
            if not resume:
                try:
                    await asyncio.shield(self.abort_multipart_upload(bucket, key, upload_id))
                except Exception:
                    pass
            raise

    async def _reusable_parts(self, bucket: str, key: str, upload_id: str, path: str,
                              parts: List[Tuple[int, int, int]]) -> Dict[int, str]:
        from ..ops import hashing
        remote = {n: (e, s) for n, e, s in await self.list_parts(bucket, key, upload_id)}
        cand = [(n, o, ln) for n, o, ln in parts if n in remote and remote[n][1] == ln]
        if not cand:
            return {}
        loop = asyncio.get_running_loop()
        md5s = await loop.run_in_executor(None, hashing.hash_file_ranges, path,
                                          [(o, ln) for _, o, ln in cand], "md5")
        return {n: remote[n][0] for (n, _, _), d in zip(cand, md5s) if d.hex() == remote[n][0]}

    # ------------------------------------------------------------------ streaming relay
    def can_relay(self, src_url: str, src_proxy=None) -> bool:
        """Socket relay source -> this endpoint possible (both http, or https with native TLS;
        an https source behind a forward proxy is not)."""
        nt = getattr(self.t, "native", None)
        proxied = src_proxy is not None and src_proxy.for_url(src_url) is not None
        return nt is not None and nt.handles(src_url, proxied) and nt.handles(self.base)

    def _signed(self, method: str, bucket: str, key: str, query: Sequence[Tuple[str, str]],
                headers: Optional[Dict[str, str]] = None,
                phash: str = sigv4.UNSIGNED) -> Tuple[str, List[Tuple[str, str]]]:
        host, path = self._address(bucket, key)
        qs = sigv4.canonical_query(query)
        url = f"{self.scheme}://{host}" + sigv4.uri_encode(path, True) + ("?" + qs if qs else "")
        hdrs = {"host": host}
        if self.session_token:
            hdrs["x-amz-security-token"] = self.session_token
        if headers:
            hdrs.update({k.lower(): v for k, v in headers.items()})
        sigv4.sign(method, path, list(query), hdrs, self.access_key, self.secret_key,
                   self.region_of(bucket), phash)
        return url, list(hdrs.items())

    async def _relay_put(self, bucket: str, key: str, query: Sequence[Tuple[str, str]],
                         src_url: str, offset: int, length: int, whole: bool,
                         progress: Optional[Progress], split=None, src_proxy=None,
                         content_type: str = "", checksum: bool = False, validator: str = "",
                         gpu: bool = False, meta: Optional[Dict[str, str]] = None):
        """One relayed PUT (object or part) with retries; returns the ETag, or with ``split``
        (see ``NativeTransport.relay``) ``(etag, {"digests", "head", "tail"})``.
        ``checksum``: aws-chunked body with a trailing CRC32C of the relayed bytes.
        ``validator``: pin the source GET to that version; a changed source raises
        ``SourceChanged`` (nothing is sent to S3 for that GET)."""
        src_hdrs = [] if whole else [("Range", f"bytes={offset}-{offset + length - 1}")]
        src_hdrs += pin_headers(validator, not whole)
        put_hdrs: Dict[str, str] = {"content-type": content_type} if content_type else {}
        put_hdrs.update({f"x-amz-meta-{k}": v for k, v in (meta or {}).items()})
        phash = sigv4.UNSIGNED
        if checksum:
            put_hdrs.update({"content-encoding": "aws-chunked",
                             "x-amz-decoded-content-length": str(length),
                             "x-amz-trailer": "x-amz-checksum-crc32c"})
            phash = sigv4.STREAMING_TRAILER
        attempt = 0
        relocated = False
        while True:
            url, hdrs = self._signed("PUT", bucket, key, query, put_hdrs or None, phash)
            try:
                get, put, _, hashed = await self.t.native.relay(src_url, src_hdrs, url, hdrs,
                                                                length, progress, split,
                                                                src_proxy=src_proxy,
                                                                checksum=checksum, gpu=gpu)
            except TransportError as e:
                err: Exception = e
                retry = True
            else:
                if put is None:
                    if get.status == 412 or (validator and not whole and get.status == 200):
                        raise SourceChanged(f"source changed since {validator} (HTTP "
                                            f"{get.status} for {length} bytes at {offset})",
                                            get.status)
                    raise TransportError(f"source {redact_url(src_url)} answered HTTP {get.status} "
                                         f"(Content-Length {get.header('content-length')}) "
                                         f"for {length} bytes at {offset}", get.status)
                if put.ok:
                    etag = PartTag.of((put.header("etag") or "").strip('"'),
                                      getattr(put, "sent_crc32c", "") if checksum else "")
                    return etag if split is None else (etag, hashed)
                hint = None if relocated else self._region_hint(put, bucket)
                if hint:
                    self._regions[bucket] = hint
                    relocated = True
                    continue
                err = parse_error(put, bucket, key)
                retry = err.retryable
            if not retry or attempt >= self.retries:
                raise err
            attempt += 1
            await asyncio.sleep(min(5.0, 0.1 * (2 ** attempt)) * (0.5 + random.random()))

    async def relay_object(self, bucket: str, key: str, src_url: str, size: int,
                           progress: Optional[Progress] = None,
                           concurrency: Optional[int] = None, src_proxy=None,
                           content_type: str = "", ranges: bool = True,
                           validator: str = "", journal: str = "",
                           keep_on_error: bool = False, stats: Optional[dict] = None,
                           meta: Optional[Dict[str, str]] = None) -> str:
        """Stage ``src_url`` (``size`` bytes) straight into S3: each multipart part is one Range
        GET relayed socket->socket into one UploadPart; objects up to ``multipart_threshold``
        go in one relayed PUT. ``src_proxy``: the source-fetch proxy policy
        (``net/proxy.ProxyConfig``); ``ranges``: the origin serves Range requests.

        ``validator`` (strong ETag or ``lm:<Last-Modified>``): every part's GET is pinned to
        that version, so parts of two versions of a changing origin are never combined into
        one object (the reference's single GET per file cannot mix versions either,
        lib/download.js:159-160). A change aborts the upload with ``SourceChanged``; the
        caller restarts from the new version.

        Over TLS one relay is bound by one thread decrypting and re-encrypting every byte
        (~2 - 3 GB/s), so with ``split_tls_relays`` an object of more than 6 MiB that would go
        in one PUT is cut into up to ``max_inflight_parts`` parts relayed in parallel.

        ``journal`` (a key in ``bucket``; multipart only, needs ``validator``): resume across
        attempts (SURVEY §5.4 "resumable multipart"). The upload id, the source version and
        the part plan are recorded there; a later call for the same object and the same
        version relays only the parts the upload does not hold yet (ListParts: same number,
        same size). ``keep_on_error``: a failure leaves the upload and its journal for that
        next attempt instead of aborting (a changed source always aborts). ``stats`` gets
        ``resumed_parts`` when parts were reused. ``meta``: user metadata (x-amz-meta-*) of
        the staged object."""
        tls = src_url.startswith("https://") or self.scheme == "https"
        crc = self.want_checksum(relay=True, tls=tls)
        if size <= self.multipart_threshold:
            if not (tls and self.split_tls_relays and ranges and size > MIN_PART + (1 << 20)):
                return await self._relay_put(bucket, key, [], src_url, 0, size, True, progress,
                                             src_proxy=src_proxy, content_type=content_type,
                                             checksum=crc, validator=validator, meta=meta)
            ps = -(-size // max(1, self.max_inflight_parts))
            parts = self.plan_parts(size, part_size=-(-ps // (1 << 20)) << 20)
        else:
            parts = self.plan_parts(size)
        journal = journal if validator else ""
        upload_id, etags = (await self._resume_relay(bucket, key, journal, validator, size,
                                                     parts) if journal else (None, {}))
        if upload_id is None:
            upload_id = await self.create_multipart_upload(bucket, key, content_type, meta,
                                                           checksum=crc)
            if journal:
                await self.put_object(bucket, journal, json.dumps(
                    {"key": key, "upload_id": upload_id, "validator": validator, "size": size,
                     "parts": [[n, o, ln] for n, o, ln in parts]}), "application/json")
        reused = len(etags)
        if progress is not None and reused:
            progress.add(sum(ln for n, _, ln in parts if n in etags))
        sem = asyncio.Semaphore(concurrency or self.max_inflight_parts)

        failed = False

        async def one(num: int, off: int, ln: int) -> None:
            async with sem:
                if failed:
                    return
                etags[num] = await self._relay_put(
                    bucket, key, [("partNumber", str(num)), ("uploadId", upload_id)], src_url,
                    off, ln, False, progress, src_proxy=src_proxy, checksum=crc,
                    validator=validator)
        tasks = [asyncio.ensure_future(one(n, o, ln)) for n, o, ln in parts if n not in etags]
        try:
            await asyncio.gather(*tasks)   # noqa: the except below settles the siblings
            etag = await self.complete_multipart_upload(bucket, key, upload_id,
                                                        [(n, etags[n]) for n, _, _ in parts])
        except BaseException as e:
            failed = True
            keep = (keep_on_error and journal and isinstance(e, Exception)
                    and not isinstance(e, SourceChanged))
            # gather() leaves the siblings of a failed part running. None may outlive this
            # call (a part landing in an upload being aborted, or after the next attempt
            # listed the parts): parts not begun are skipped; those in flight finish when
            # the upload is kept (the next attempt reuses them), else they are cancelled.
            if not keep:
                for t in tasks:
                    t.cancel()
            await drain(tasks)
            if not keep:
                try:
                    await asyncio.shield(self.abort_multipart_upload(bucket, key, upload_id))
                    if journal:
                        await asyncio.shield(self.delete_object(bucket, journal))
                except Exception:
                    pass
            raise
        self.resumed_parts += reused
        if stats is not None and reused:
            stats["resumed_parts"] = stats.get("resumed_parts", 0) + reused
        if journal:
            try:
                await self.delete_object(bucket, journal)
            except Exception:
                pass
        return etag

    async def _resume_relay(self, bucket: str, key: str, journal: str, validator: str,
                            size: int, parts) -> Tuple[Optional[str], Dict[int, str]]:
        """(upload id, {part: etag} already held) from a previous attempt's journal, or
        (None, {}) to start fresh - the journal missing, for another object, version, size or
        part plan, or its upload gone. Parts count only with the planned size and an ETag."""
        try:
            j = json.loads(await self.get_object(bucket, journal))
        except (S3Error, ValueError):
            return None, {}
        plan = [[n, o, ln] for n, o, ln in parts]
        if not isinstance(j, dict) or not j.get("upload_id"):
            return None, {}
        if j.get("key") != key or j.get("validator") != validator or j.get("size") != size \
                or j.get("parts") != plan:
            # another version (or plan): its parts are useless - do not leave them behind
            try:
                await self.abort_multipart_upload(bucket, j.get("key") or key, j["upload_id"])
            except Exception:
                pass
            return None, {}
        try:
            held = await self.list_parts(bucket, key, j["upload_id"])
        except S3Error:
            return None, {}
        want = {n: ln for n, _, ln in parts}
        return j["upload_id"], {n: PartTag.of(e.strip('"'), getattr(e, "crc32c", ""))
                                for n, e, sz in held
                                if want.get(n) == sz and e}

    async def copy_object(self, src_bucket: str, src_key: str, bucket: str, key: str, size: int,
                          content_type: str = "", concurrency: Optional[int] = None) -> str:
        """Server-side copy (no bytes through this process): CopyObject up to 5 GiB, above
        that a multipart upload of UploadPartCopy ranges in parallel. Both buckets must be on
        this endpoint and readable / writable with these credentials."""
        source = "/" + sigv4.uri_encode(f"{src_bucket}/{src_key}", True)
        if size <= COPY_MAX:
            hdrs = {"x-amz-copy-source": source, "x-amz-metadata-directive": "REPLACE",
                    "content-type": content_type or "application/octet-stream"}
            r = await self._request("PUT", bucket, key, headers=hdrs)
            return self._copy_etag(r, bucket, key)
        parts = self.plan_parts(size, part_size=max(self.part_size, COPY_PART))
        upload_id = await self.create_multipart_upload(bucket, key, content_type)
        sem = asyncio.Semaphore(concurrency or self.max_inflight_parts)
        etags: Dict[int, str] = {}

        async def one(num: int, off: int, ln: int) -> None:
            async with sem:
                r = await self._request(
                    "PUT", bucket, key, [("partNumber", str(num)), ("uploadId", upload_id)],
                    headers={"x-amz-copy-source": source,
                             "x-amz-copy-source-range": f"bytes={off}-{off + ln - 1}"})
                etags[num] = self._copy_etag(r, bucket, key)
        try:
            await gather_strict(*(one(n, o, ln) for n, o, ln in parts))
            return await self.complete_multipart_upload(bucket, key, upload_id,
                                                        [(n, etags[n]) for n, _, _ in parts])
        except BaseException:
            try:
                await asyncio.shield(self.abort_multipart_upload(bucket, key, upload_id))
            except Exception:
                pass
            raise

    @staticmethod
    def _copy_etag(r: Response, bucket: str, key: str) -> str:
        """ETag of a CopyObject / UploadPartCopy reply - which S3 may send as 200 with an
        <Error> body when the copy fails after the headers went out."""
        try:
            root = ET.fromstring(r.body)
        except ET.ParseError as e:
            raise S3Error("InvalidResponse", f"copy reply: {e}", r.status, key, bucket) from e
        if root.tag.split("}")[-1] == "Error":
            raise S3Error(_text(root, "Code") or "InternalError", _text(root, "Message"),
                          r.status, key, bucket)
        return _text(root, "ETag").strip('"')

    async def relay_hashed(self, bucket: str, key: str, src_url: str, offset: int, length: int,
                           whole: bool, split: Tuple[int, int, int],
                           part: Optional[Tuple[int, str]] = None,
                           progress: Optional[Progress] = None, content_type: str = "",
                           gpu: bool = False):
        """Relay ``length`` bytes of ``src_url`` at ``offset`` into the object ``key`` (or its
        multipart ``part=(number, upload_id)``) while SHA-1-ing the torrent pieces inside it
        (``split``); returns ``(etag, {"digests", "head", "tail", "gpu_ticket"})`` - with
        ``gpu`` the pieces may be queued to the part hasher instead (``gpu_ticket`` != 0)."""
        query = [] if part is None else [("partNumber", str(part[0])), ("uploadId", part[1])]
        tls = src_url.startswith("https://") or self.scheme == "https"
        return await self._relay_put(bucket, key, query, src_url, offset, length, whole,
                                     progress, split,
                                     content_type=content_type if part is None else "",
                                     checksum=self.want_checksum(relay=True, tls=tls,
                                                                 hashed=True), gpu=gpu)

    async def create_multipart_upload(self, bucket: str, key: str, content_type: str = "",
                                      meta: Optional[Dict[str, str]] = None,
                                      checksum: bool = False) -> str:
        """``checksum``: the parts will carry x-amz-checksum-crc32c - declared here
        (x-amz-checksum-algorithm), since S3 refuses part checksums of a type the upload was
        not created with."""
        hdrs = {"content-type": content_type} if content_type else {}
        if checksum:
            hdrs["x-amz-checksum-algorithm"] = "CRC32C"
        hdrs.update({f"x-amz-meta-{k}": v for k, v in (meta or {}).items()})
        r = await self._request("POST", bucket, key, query=[("uploads", "")],
                                headers=hdrs or None)
        return _text(ET.fromstring(r.body), "UploadId")

    async def upload_part(self, bucket: str, key: str, upload_id: str, num: int, body,
                          progress: Optional[Progress] = None) -> str:
        ck = self.want_checksum()
        r = await self._request("PUT", bucket, key,
                                query=[("partNumber", str(num)), ("uploadId", upload_id)],
                                body=body, progress=progress, checksum=ck)
        return PartTag.of((r.header("etag") or "").strip('"'),
                          (r.sent_checksum if ck else "") or "")

    async def complete_multipart_upload(self, bucket: str, key: str, upload_id: str,
                                        parts: Sequence[Tuple[int, str]]) -> str:
        """CompleteMultipartUpload. A lost reply makes the transport retry, and the retry
        answers NoSuchUpload because the first attempt DID complete: then the object's
        multipart ETag ("<md5 of part md5s>-<n>") is checked against the parts sent, and a
        match counts as success instead of failing a job whose object is in place."""
        xml = "".join(f"<Part><PartNumber>{n}</PartNumber><ETag>\"{e}\"</ETag>"
                      + (f"<ChecksumCRC32C>{e.crc32c}</ChecksumCRC32C>"
                         if getattr(e, "crc32c", "") else "") + "</Part>"
                      for n, e in parts)
        body = f"<CompleteMultipartUpload>{xml}</CompleteMultipartUpload>".encode()
        try:
            r = await self._request("POST", bucket, key, query=[("uploadId", upload_id)],
                                    body=body)
        except S3Error as e:
            if e.code != "NoSuchUpload":
                raise
            try:
                info = await self.head_object(bucket, key)
            except S3Error:
                raise e from None
            try:
                want = multipart_etag([t for _, t in parts])
            except ValueError:      # part ETags that are not MD5 hex (SSE-KMS / SSE-C, ...)
                raise e from None
            if info.etag != want:
                raise
            return info.etag
        root = ET.fromstring(r.body)
        if _strip(root.tag) == "Error":
            raise S3Error(_text(root, "Code"), _text(root, "Message"), 200, key, bucket)
        return _text(root, "ETag").strip('"')

    async def abort_multipart_upload(self, bucket: str, key: str, upload_id: str) -> None:
        await self._request("DELETE", bucket, key, query=[("uploadId", upload_id)], ok=(404,))

    async def list_parts(self, bucket: str, key: str, upload_id: str) -> List[Tuple[int, str, int]]:
        out: List[Tuple[int, str, int]] = []
        marker = ""
        while True:
            q = [("uploadId", upload_id)] + ([("part-number-marker", marker)] if marker else [])
            r = await self._request("GET", bucket, key, query=q)
            root = ET.fromstring(r.body)
            for p in root:
                if _strip(p.tag) == "Part":
                    out.append((int(_text(p, "PartNumber")),
                                PartTag.of(_text(p, "ETag").strip('"'),
                                           _text(p, "ChecksumCRC32C")),
                                int(_text(p, "Size", "0"))))
            if _text(root, "IsTruncated") != "true":
                return out
            marker = _text(root, "NextPartNumberMarker")

    async def list_uploads(self, bucket: str, prefix: str,
                           page: int = 1000) -> List[Tuple[str, str]]:
        """(key, upload id) of every multipart upload in progress under ``prefix``
        (ListMultipartUploads, paginated by key / upload-id marker)."""
        out: List[Tuple[str, str]] = []
        km = um = ""
        while True:
            q = [("uploads", ""), ("prefix", prefix), ("max-uploads", str(page))]
            if km:
                q += [("key-marker", km), ("upload-id-marker", um)]
            r = await self._request("GET", bucket, query=q)
            root = ET.fromstring(r.body)
            for u in root:
                if _strip(u.tag) == "Upload":
                    out.append((_text(u, "Key"), _text(u, "UploadId")))
            nk, nu = _text(root, "NextKeyMarker"), _text(root, "NextUploadIdMarker")
            if _text(root, "IsTruncated") != "true" or not nk or (nk, nu) == (km, um):
                return out
            km, um = nk, nu

    async def find_upload(self, bucket: str, key: str) -> Optional[str]:
        """Upload id of an upload in progress for exactly ``key`` (the last listed)."""
        best = None
        for k, uid in await self.list_uploads(bucket, key):
            if k == key:
                best = uid
        return best

    async def fget_object(self, bucket: str, key: str, path: str, streams: int = 1,
                          min_split: int = 32 * MiB, progress: Optional[Progress] = None) -> int:
        """Download to ``path`` (via ``path + '.part'`` then rename, like minio-js)."""
        tmp = path + ".part"
        os.makedirs(os.path.dirname(os.path.abspath(path)) or ".", exist_ok=True)
        fd = os.open(tmp, os.O_WRONLY | os.O_CREAT | os.O_TRUNC | getattr(os, "O_CLOEXEC", 0),
                     0o644)
        try:
            size = -1
            if streams > 1:
                size = (await self.head_object(bucket, key)).size
            if streams > 1 and size >= 2 * min_split:
                os.ftruncate(fd, size)
                n = min(streams, max(1, size // min_split))
                step = (size + n - 1) // n
                rngs = [(o, min(step, size - o)) for o in range(0, size, step)]

                async def one(off: int, ln: int) -> None:
                    await self._request("GET", bucket, key,
                                        headers={"range": f"bytes={off}-{off + ln - 1}"},
                                        sink=FileSink(fd, off, ln), progress=progress)
                await gather_strict(*(one(o, ln) for o, ln in rngs))
                written = size
            else:
                r = await self._request("GET", bucket, key, sink=FileSink(fd, 0),
                                        progress=progress)
                written = r.written
        finally:
            os.close(fd)
        os.replace(tmp, path)
        return written

    async def list_objects(self, bucket: str, prefix: str = "", recursive: bool = True,
                           max_keys: int = 1000) -> List[ObjectInfo]:
        """ListObjectsV2 with pagination (``getObjects`` in triton-core/minio)."""
        out: List[ObjectInfo] = []
        token = ""
        while True:
            q = [("list-type", "2"), ("prefix", prefix), ("max-keys", str(max_keys))]
            if not recursive:
                q.append(("delimiter", "/"))
            if token:
                q.append(("continuation-token", token))
            r = await self._request("GET", bucket, query=q)
            root = ET.fromstring(r.body)
            for c in root:
                t = _strip(c.tag)
                if t == "Contents":
                    out.append(ObjectInfo(_text(c, "Key"), int(_text(c, "Size", "0")),
                                          _text(c, "ETag").strip('"'), _text(c, "LastModified")))
                elif t == "CommonPrefixes":
                    out.append(ObjectInfo(_text(c, "Prefix"), 0))
            if _text(root, "IsTruncated") != "true":
                return out
            token = _text(root, "NextContinuationToken")
            if not token:    # truncated without a continuation token: would loop forever
                raise S3Error("InvalidResponse", "IsTruncated without NextContinuationToken",
                              200, "", bucket)


class PartTag(str):
    """A part's ETag that also carries the CRC32C it was uploaded with (base64, "" = none):
    CompleteMultipartUpload lists it as <ChecksumCRC32C> when the upload declared CRC32C."""
    crc32c = ""

    @classmethod
    def of(cls, etag: str, crc32c: str = "") -> "PartTag":
        t = cls(etag)
        t.crc32c = crc32c or ""
        return t


def multipart_etag(part_etags: Sequence[str]) -> str:
    """S3's ETag of a completed multipart object: MD5 of the concatenated binary part MD5s,
    then ``-<part count>``."""
    import hashlib
    md5s = b"".join(bytes.fromhex(e.strip('"')) for e in part_etags)
    return f"{hashlib.md5(md5s).hexdigest()}-{len(part_etags)}"


def object_url_path(bucket: str, key: str) -> str:
    return "/" + quote(bucket) + "/" + quote(key, safe="/-_.~")


ProgressCb = Callable[[int], None]
