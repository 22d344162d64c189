"""In-process S3-compatible server for tests (MinIO stand-in; no MinIO binary in the image).

Implements the subset the stager and the ``bucket://`` source use: bucket HEAD/PUT/DELETE,
ListObjectsV2 (prefix, delimiter, continuation), object PUT/GET (Range)/HEAD/DELETE, multipart
(initiate, upload part, complete, abort, list parts, list uploads). Requests are SigV4
verified (``x-amz-content-sha256`` too unless UNSIGNED-PAYLOAD). ETags are MD5 / multipart
``md5(concat(part md5s))-N`` like S3.

Fault injection: ``faults.add(FaultRule(...))`` makes matching requests fail
with a status/code, stall, or drop the connection mid-response.

Payload integrity like S3: ``x-amz-checksum-crc32c`` (header, or trailer of an aws-chunked
body with ``x-amz-content-sha256: STREAMING-UNSIGNED-PAYLOAD-TRAILER``) and ``Content-MD5`` are
recomputed over the received bytes; a mismatch is 400 BadDigest and nothing is stored.
``corrupt_next = n`` flips one byte of the next n checksummed PUT bodies on arrival (transit
corruption the checksum must catch).
"""
from __future__ import annotations

import asyncio
import base64
import hashlib
import secrets
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional, Tuple
from urllib.parse import parse_qsl, unquote
from xml.sax.saxutils import escape

from aiohttp import web

from . import sigv4

XMLNS = "http://s3.amazonaws.com/doc/2006-03-01/"


@dataclass
class StoredObject:
    data: bytes
    etag: str
    mtime: float = field(default_factory=time.time)
    content_type: str = "application/octet-stream"
    meta: Dict[str, str] = field(default_factory=dict)     # x-amz-meta-* (user metadata)


@dataclass
class Upload:
    key: str
    content_type: str = "application/octet-stream"
    parts: Dict[int, Tuple[bytes, str]] = field(default_factory=dict)
    initiated: float = field(default_factory=time.time)
    meta: Dict[str, str] = field(default_factory=dict)
    # x-amz-checksum-algorithm declared at CreateMultipartUpload ("" = none): a part that
    # carries another checksum type is refused, as S3 does ("Checksum Type mismatch")
    algorithm: str = ""
    crcs: Dict[int, str] = field(default_factory=dict)      # part -> its CRC32C (base64)


def _user_meta(headers) -> Dict[str, str]:
    return {k.lower(): v for k, v in headers.items() if k.lower().startswith("x-amz-meta-")}


@dataclass
class FaultRule:
    method: str = "*"
    path_contains: str = ""
    query_contains: str = ""
    times: int = 1
    status: int = 503
    code: str = "SlowDown"
    delay_s: float = 0.0
    drop_connection: bool = False
    # process the request, then drop the connection before the response (a lost reply:
    # the client cannot tell whether e.g. CompleteMultipartUpload happened)
    drop_after: bool = False

    def matches(self, method: str, path: str, query: str) -> bool:
        return ((self.method == "*" or self.method == method)
                and self.path_contains in path and self.query_contains in query)


class Faults:
    def __init__(self) -> None:
        self.rules: List[FaultRule] = []
        self.fired: List[Tuple[str, str]] = []
        self._lock = threading.Lock()

    def add(self, rule: FaultRule) -> None:
        with self._lock:
            self.rules.append(rule)

    def take(self, method: str, path: str, query: str) -> Optional[FaultRule]:
        with self._lock:
            for r in self.rules:
                if r.times > 0 and r.matches(method, path, query):
                    r.times -= 1
                    self.fired.append((method, path))
                    return r
        return None


def decode_aws_chunked(body: bytes) -> Optional[Tuple[bytes, Dict[str, str]]]:
    """``(payload, trailers)`` of an aws-chunked body (``<hex>[;ext]\r\n<data>\r\n`` ...
    ``0\r\n<trailer lines>\r\n``), or None when malformed."""
    out, pos, trailers = [], 0, {}
    while True:
        e = body.find(b"\r\n", pos)
        if e < 0:
            return None
        try:
            n = int(body[pos:e].split(b";", 1)[0], 16)
        except ValueError:
            return None
        pos = e + 2
        if n == 0:
            while True:
                e = body.find(b"\r\n", pos)
                if e < 0:
                    return None
                line = body[pos:e].decode("latin-1")
                pos = e + 2
                if not line:
                    return b"".join(out), trailers
                k, _, v = line.partition(":")
                trailers[k.strip().lower()] = v.strip()
        if pos + n + 2 > len(body) or body[pos + n:pos + n + 2] != b"\r\n":
            return None
        out.append(body[pos:pos + n])
        pos += n + 2


def _xml(body: str) -> web.Response:
    return web.Response(body=('<?xml version="1.0" encoding="UTF-8"?>' + body).encode(),
                        content_type="application/xml")


def _err(status: int, code: str, msg: str = "", resource: str = "") -> web.Response:
    return web.Response(status=status, content_type="application/xml", body=(
        f'<?xml version="1.0" encoding="UTF-8"?><Error><Code>{code}</Code>'
        f"<Message>{escape(msg or code)}</Message><Resource>{escape(resource)}</Resource>"
        f"<RequestId>{secrets.token_hex(8)}</RequestId></Error>").encode())


class FakeS3:
    def __init__(self, access_key: str = "minioadmin", secret_key: str = "minioadmin",
                 verify_signatures: bool = True, host: str = "127.0.0.1", port: int = 0,
                 ssl_context=None, virtual_host_suffix: str = ""):
        self.creds = {access_key: secret_key}
        self.verify_signatures = verify_signatures
        self.buckets: Dict[str, Dict[str, StoredObject]] = {}
        self.uploads: Dict[str, Dict[str, Upload]] = {}
        self.faults = Faults()
        self.requests: List[Tuple[str, str]] = []
        self.host = host
        self.port = port
        self._runner: Optional[web.AppRunner] = None
        self._thread: Optional[threading.Thread] = None
        self._loop: Optional[asyncio.AbstractEventLoop] = None
        self.hooks: List[Callable[[str, str], None]] = []
        self.ssl_context = ssl_context          # serve https (tests of secure / bucket://)
        # virtual-hosted-style requests: Host "<bucket>.<suffix>[:port]", path "/<key>"
        self.virtual_host_suffix = virtual_host_suffix
        # bucket -> region: requests signed for another region are refused the way AWS does
        # (400 AuthorizationHeaderMalformed + x-amz-bucket-region)
        self.bucket_regions: Dict[str, str] = {}
        # access key -> session token it must present (signed) as x-amz-security-token
        self.session_tokens: Dict[str, str] = {}
        self.server_copies = 0                  # CopyObject / UploadPartCopy served
        self.corrupt_next = 0                   # flip a byte of the next n checksummed PUTs
        self.corrupted = 0
        self.bad_digests = 0                    # PUTs refused: payload checksum mismatch
        self.checksummed = 0                    # PUTs that carried a payload checksum
        self.checksum_type_mismatches = 0       # parts refused: checksum type not declared
        self.complete_part_checksums = 0        # <ChecksumCRC32C> checked at Complete

    # ---------------------------------------------------------------- lifecycle
    @property
    def endpoint(self) -> str:
        return f"{self.host}:{self.port}"

    async def start(self) -> str:
        app = web.Application(client_max_size=1 << 40)
        app.router.add_route("*", "/{tail:.*}", self._handle)
        self._runner = web.AppRunner(app, access_log=None)
        await self._runner.setup()
        site = web.TCPSite(self._runner, self.host, self.port, ssl_context=self.ssl_context)
        await site.start()
        self.port = site._server.sockets[0].getsockname()[1]  # type: ignore[union-attr]
        return self.endpoint

    async def stop(self) -> None:
        if self._runner is not None:
            await self._runner.cleanup()
            self._runner = None

    def start_in_thread(self) -> str:
        ready = threading.Event()

        def run() -> None:
            self._loop = asyncio.new_event_loop()
            asyncio.set_event_loop(self._loop)
            self._loop.run_until_complete(self.start())
            ready.set()
            self._loop.run_forever()
            self._loop.run_until_complete(self.stop())
            self._loop.close()

        self._thread = threading.Thread(target=run, daemon=True, name="fake-s3")
        self._thread.start()
        ready.wait(30)
        return self.endpoint

    def stop_thread(self) -> None:
        if self._loop is not None:
            self._loop.call_soon_threadsafe(self._loop.stop)
        if self._thread is not None:
            self._thread.join(10)

    # ---------------------------------------------------------------- helpers for tests
    def objects(self, bucket: str) -> Dict[str, StoredObject]:
        return self.buckets.get(bucket, {})

    def get(self, bucket: str, key: str) -> Optional[bytes]:
        o = self.buckets.get(bucket, {}).get(key)
        return None if o is None else o.data

    def put(self, bucket: str, key: str, data: bytes) -> None:
        self.buckets.setdefault(bucket, {})[key] = StoredObject(data, hashlib.md5(data).hexdigest())

    # ---------------------------------------------------------------- dispatch
    async def _handle(self, req: web.Request) -> web.StreamResponse:
        raw_path, _, raw_query = req.raw_path.partition("?")
        path = sig_path = unquote(raw_path)
        query = parse_qsl(raw_query, keep_blank_values=True)
        vb = self._virtual_bucket(req.headers.get("Host", ""))
        if vb:
            path = "/" + vb + (path if path != "/" else "")
        self.requests.append((req.method, path))
        for h in self.hooks:
            h(req.method, path)
        rule = self.faults.take(req.method, path, raw_query)
        if rule is not None:
            if rule.delay_s:
                await asyncio.sleep(rule.delay_s)
            if rule.drop_connection:
                if req.transport is not None:
                    req.transport.close()
                raise web.HTTPInternalServerError()
            if rule.status and not rule.drop_after:
                return _err(rule.status, rule.code, "injected fault", path)
        resp = await self._dispatch(req, path, query, sig_path)
        if rule is not None and rule.drop_after:
            if req.transport is not None:
                req.transport.close()
            raise web.HTTPInternalServerError()
        return resp

    def _virtual_bucket(self, host: str) -> str:
        sfx = self.virtual_host_suffix
        name = host.rsplit(":", 1)[0] if host.count(":") == 1 else host
        if sfx and name.endswith("." + sfx):
            return name[:-len(sfx) - 1]
        return ""

    def _check_payload(self, req: web.Request, body: bytes, trailers: Dict[str, str],
                       path: str):
        """S3 payload checksums of a PUT; returns (possibly corrupted) body, the CRC header to
        echo, and an error response or None."""
        from ..ops import hashing
        want_crc = req.headers.get("x-amz-checksum-crc32c") or trailers.get("x-amz-checksum-crc32c")
        want_md5 = req.headers.get("Content-MD5")
        if "x-amz-checksum-crc32c" in req.headers.get("x-amz-trailer", "") and \
                "x-amz-checksum-crc32c" not in trailers:
            return body, "", _err(400, "MalformedTrailerError", "declared trailer missing", path)
        if want_crc is None and want_md5 is None:
            return body, "", None
        self.checksummed += 1
        if self.corrupt_next > 0 and body:
            self.corrupt_next -= 1
            self.corrupted += 1
            i = len(body) // 2
            body = body[:i] + bytes([body[i] ^ 0x01]) + body[i + 1:]
        if want_crc is not None and hashing.crc32c_b64(body) != want_crc:
            self.bad_digests += 1
            return body, "", _err(400, "BadDigest", "The CRC32C you specified did not match "
                                  "the calculated checksum.", path)
        if want_md5 is not None and \
                base64.b64encode(hashlib.md5(body).digest()).decode() != want_md5:
            self.bad_digests += 1
            return body, "", _err(400, "BadDigest", "The Content-MD5 you specified did not "
                                  "match what was received.", path)
        return body, want_crc or "", None

    async def _dispatch(self, req: web.Request, path: str, query,
                        sig_path: str = "") -> web.StreamResponse:
        body = await req.read() if req.can_read_body else b""
        trailers: Dict[str, str] = {}
        if "aws-chunked" in req.headers.get("Content-Encoding", ""):
            dec = decode_aws_chunked(body)
            want_len = req.headers.get("x-amz-decoded-content-length", "")
            if dec is None or not want_len.isdigit() or int(want_len) != len(dec[0]):
                return _err(400, "IncompleteBody", "bad aws-chunked body", path)
            body, trailers = dec
        presigned = any(k == "X-Amz-Signature" for k, _ in query)
        presigned_cred = dict(query).get("X-Amz-Credential", "")
        if self.verify_signatures and presigned:
            hdrs = {k.lower(): v for k, v in req.headers.items()}
            ok, reason = sigv4.verify_presigned(req.method, sig_path or path, query, hdrs,
                                                self.creds)
            if not ok:
                return _err(403, reason, "presigned URL check failed", path)
            query = [(k, v) for k, v in query if not k.startswith("X-Amz-")]
        elif self.verify_signatures:
            hdrs = {k.lower(): v for k, v in req.headers.items()}
            ok, reason = sigv4.verify(req.method, sig_path or path, query, hdrs, self.creds)
            if not ok:
                return _err(403, reason, "signature check failed", path)
            if self.session_tokens:
                auth = sigv4.parse_authorization(hdrs["authorization"])
                tok = self.session_tokens.get(auth["Credential"].split("/")[0])
                if tok is not None and (hdrs.get("x-amz-security-token") != tok or
                                        "x-amz-security-token" not in
                                        auth["SignedHeaders"].split(";")):
                    return _err(403, "InvalidToken", "missing or bad session token", path)
            ph = hdrs.get("x-amz-content-sha256", "")
            if ph not in (sigv4.UNSIGNED, sigv4.STREAMING_TRAILER) and \
                    ph != hashlib.sha256(body).hexdigest():
                return _err(400, "XAmzContentSHA256Mismatch", "", path)
            if ph == sigv4.STREAMING_TRAILER and not trailers:
                return _err(400, "IncompleteBody", "streaming payload without trailer", path)
        echo = ""
        if req.method == "PUT":
            body, echo, bad = self._check_payload(req, body, trailers, path)
            if bad is not None:
                return bad
        want = self.bucket_regions.get(path.lstrip("/").split("/", 1)[0])
        if want:
            try:
                cred = presigned_cred if presigned else \
                    sigv4.parse_authorization(req.headers.get("Authorization", ""))["Credential"]
                got = cred.split("/")[2]
            except (ValueError, KeyError, IndexError, AttributeError):
                got = ""
            if got != want:
                r = _err(400, "AuthorizationHeaderMalformed",
                         f"the region '{got}' is wrong; expecting '{want}'", path)
                r.body = r.body.replace(b"</Error>", f"<Region>{want}</Region></Error>".encode())
                r.headers["x-amz-bucket-region"] = want
                return r
        parts = path.lstrip("/").split("/", 1)
        bucket = parts[0]
        key = parts[1] if len(parts) > 1 else ""
        q = dict(query)
        if not bucket:
            return self._list_buckets()
        if not key:
            return self._bucket_op(req.method, bucket, q)
        resp = self._object_op(req, bucket, key, q, body, echo)
        if echo and resp.status == 200:
            resp.headers["x-amz-checksum-crc32c"] = echo
        return resp

    def _copy_source(self, src: str, rng: Optional[str]):
        """Bytes named by ``x-amz-copy-source: /bucket/key`` (URL-encoded), optionally
        ``x-amz-copy-source-range: bytes=a-b``; an error response when missing."""
        sb, _, sk = unquote(src).lstrip("/").partition("/")
        obj = self.buckets.get(sb, {}).get(sk)
        if obj is None:
            return _err(404, "NoSuchKey", "copy source", src)
        if not rng:
            return obj.data
        try:
            a, b = rng.split("=", 1)[1].split("-")
            a, b = int(a), int(b)
        except (IndexError, ValueError):
            return _err(400, "InvalidArgument", "bad copy source range", src)
        if not 0 <= a <= b < len(obj.data):
            return _err(416, "InvalidRange", "", src)
        return obj.data[a:b + 1]

    def _list_buckets(self) -> web.Response:
        b = "".join(f"<Bucket><Name>{escape(n)}</Name></Bucket>" for n in sorted(self.buckets))
        return _xml(f'<ListAllMyBucketsResult xmlns="{XMLNS}"><Buckets>{b}</Buckets>'
                    "</ListAllMyBucketsResult>")

    def _bucket_op(self, method: str, bucket: str, q: Dict[str, str]) -> web.Response:
        exists = bucket in self.buckets
        if method == "HEAD":
            return web.Response(status=200 if exists else 404)
        if method == "PUT":
            if exists:
                return _err(409, "BucketAlreadyOwnedByYou", "", bucket)
            self.buckets[bucket] = {}
            self.uploads[bucket] = {}
            return web.Response(status=200)
        if not exists:
            return _err(404, "NoSuchBucket", "", bucket)
        if method == "DELETE":
            if self.buckets[bucket]:
                return _err(409, "BucketNotEmpty", "", bucket)
            del self.buckets[bucket]
            return web.Response(status=204)
        if method == "GET" and "uploads" in q:
            # ListMultipartUploads, sorted by (key, upload id) and paginated like S3
            # (max-uploads, key-marker / upload-id-marker -> NextKeyMarker / NextUploadIdMarker)
            prefix = q.get("prefix", "")
            limit = max(1, min(1000, int(q.get("max-uploads", "1000") or 1000)))
            marker = (q.get("key-marker", ""), q.get("upload-id-marker", ""))
            allu = sorted((u.key, uid) for uid, u in self.uploads.get(bucket, {}).items()
                          if u.key.startswith(prefix))
            if marker[0]:
                allu = [ku for ku in allu if ku > marker]
            page, more = allu[:limit], len(allu) > limit
            ups = "".join(f"<Upload><Key>{escape(k)}</Key><UploadId>{uid}</UploadId></Upload>"
                          for k, uid in page)
            nxt = (f"<NextKeyMarker>{escape(page[-1][0])}</NextKeyMarker>"
                   f"<NextUploadIdMarker>{page[-1][1]}</NextUploadIdMarker>") if more else ""
            return _xml(f'<ListMultipartUploadsResult xmlns="{XMLNS}"><Bucket>{bucket}</Bucket>'
                        f"<IsTruncated>{'true' if more else 'false'}</IsTruncated>{nxt}"
                        f"{ups}</ListMultipartUploadsResult>")
        if method == "GET":
            return self._list_v2(bucket, q)
        return _err(405, "MethodNotAllowed", "", bucket)

    def _list_v2(self, bucket: str, q: Dict[str, str]) -> web.Response:
        prefix = q.get("prefix", "")
        delim = q.get("delimiter", "")
        max_keys = int(q.get("max-keys", "1000"))
        start = q.get("continuation-token", "") or q.get("start-after", "")
        keys = sorted(k for k in self.buckets[bucket] if k.startswith(prefix) and k > start)
        contents, prefixes = [], []
        seen = set()
        last = ""
        truncated = False
        for k in keys:
            if len(contents) + len(prefixes) >= max_keys:
                truncated = True
                break
            if delim:
                rest = k[len(prefix):]
                if delim in rest:
                    cp = prefix + rest.split(delim, 1)[0] + delim
                    if cp not in seen:
                        seen.add(cp)
                        prefixes.append(cp)
                    last = k
                    continue
            o = self.buckets[bucket][k]
            contents.append(f"<Contents><Key>{escape(k)}</Key><Size>{len(o.data)}</Size>"
                            f"<ETag>&quot;{o.etag}&quot;</ETag><LastModified>"
                            f"{time.strftime('%Y-%m-%dT%H:%M:%S.000Z', time.gmtime(o.mtime))}"
                            f"</LastModified><StorageClass>STANDARD</StorageClass></Contents>")
            last = k
        cps = "".join(f"<CommonPrefixes><Prefix>{escape(p)}</Prefix></CommonPrefixes>"
                      for p in prefixes)
        nxt = f"<NextContinuationToken>{escape(last)}</NextContinuationToken>" if truncated else ""
        return _xml(f'<ListBucketResult xmlns="{XMLNS}"><Name>{bucket}</Name>'
                    f"<Prefix>{escape(prefix)}</Prefix><KeyCount>{len(contents)}</KeyCount>"
                    f"<MaxKeys>{max_keys}</MaxKeys><IsTruncated>{str(truncated).lower()}"
                    f"</IsTruncated>{nxt}{''.join(contents)}{cps}</ListBucketResult>")

    def _object_op(self, req: web.Request, bucket: str, key: str, q: Dict[str, str],
                   body: bytes, crc: str = "") -> web.Response:
        if bucket not in self.buckets:
            return _err(404, "NoSuchBucket", "", bucket)
        objs = self.buckets[bucket]
        ups = self.uploads.setdefault(bucket, {})
        m = req.method
        if m == "POST" and "uploads" in q:
            uid = secrets.token_hex(16)
            algo = req.headers.get("x-amz-checksum-algorithm", "").upper()
            if algo and algo not in ("CRC32C", "CRC32", "SHA1", "SHA256"):
                return _err(400, "InvalidRequest", f"bad checksum algorithm {algo}", key)
            ups[uid] = Upload(key, req.headers.get("Content-Type", "application/octet-stream"),
                              meta=_user_meta(req.headers), algorithm=algo)
            return _xml(f'<InitiateMultipartUploadResult xmlns="{XMLNS}"><Bucket>{bucket}</Bucket>'
                        f"<Key>{escape(key)}</Key><UploadId>{uid}</UploadId>"
                        "</InitiateMultipartUploadResult>")
        if "uploadId" in q:
            up = ups.get(q["uploadId"])
            if up is None or up.key != key:
                return _err(404, "NoSuchUpload", "", key)
            if m == "PUT":
                num = int(q.get("partNumber", "0"))
                if not 1 <= num <= 10000:
                    return _err(400, "InvalidArgument", "bad part number", key)
                src = req.headers.get("x-amz-copy-source")
                if src:                              # UploadPartCopy
                    data = self._copy_source(src, req.headers.get("x-amz-copy-source-range"))
                    if isinstance(data, web.Response):
                        return data
                    etag = hashlib.md5(data).hexdigest()
                    up.parts[num] = (data, etag)
                    self.server_copies += 1
                    return _xml(f'<CopyPartResult xmlns="{XMLNS}"><ETag>&quot;{etag}&quot;</ETag>'
                                "</CopyPartResult>")
                if crc and up.algorithm != "CRC32C":
                    self.checksum_type_mismatches += 1
                    return _err(400, "InvalidRequest", "Checksum Type mismatch occurred, "
                                f"expected checksum Type: {up.algorithm.lower() or 'null'}, "
                                "actual checksum Type: crc32c", key)
                etag = hashlib.md5(body).hexdigest()
                up.parts[num] = (body, etag)
                if crc:
                    up.crcs[num] = crc
                else:
                    up.crcs.pop(num, None)
                return web.Response(status=200, headers={"ETag": f'"{etag}"'})
            if m == "GET":
                ps = "".join(f"<Part><PartNumber>{n}</PartNumber><ETag>&quot;{e}&quot;</ETag>"
                             + (f"<ChecksumCRC32C>{up.crcs[n]}</ChecksumCRC32C>"
                                if n in up.crcs else "")
                             + f"<Size>{len(d)}</Size></Part>"
                             for n, (d, e) in sorted(up.parts.items()))
                return _xml(f'<ListPartsResult xmlns="{XMLNS}"><Bucket>{bucket}</Bucket>'
                            f"<Key>{escape(key)}</Key><UploadId>{q['uploadId']}</UploadId>"
                            f"<IsTruncated>false</IsTruncated>{ps}</ListPartsResult>")
            if m == "DELETE":
                del ups[q["uploadId"]]
                return web.Response(status=204)
            if m == "POST":
                import xml.etree.ElementTree as ET
                try:
                    root = ET.fromstring(body)
                except ET.ParseError:
                    return _err(400, "MalformedXML", "", key)
                want = []
                for p in root:
                    n = e = None
                    ck = None
                    for c in p:
                        t = c.tag.split("}")[-1]
                        if t == "PartNumber":
                            n = int(c.text or 0)
                        elif t == "ETag":
                            e = (c.text or "").strip('"')
                        elif t == "ChecksumCRC32C":
                            ck = (c.text or "").strip()
                    # a part checksum in Complete must be the one the part was stored with
                    if ck is not None and (up.algorithm != "CRC32C" or up.crcs.get(n) != ck):
                        return _err(400, "InvalidPart", f"part {n}: checksum", key)
                    if ck is not None:
                        self.complete_part_checksums += 1
                    want.append((n, e))
                if [n for n, _ in want] != sorted(n for n, _ in want):
                    return _err(400, "InvalidPartOrder", "", key)
                datas, md5s = [], b""
                for i, (n, e) in enumerate(want):
                    got = up.parts.get(n)
                    if got is None or got[1] != e:
                        return _err(400, "InvalidPart", f"part {n}", key)
                    if i < len(want) - 1 and len(got[0]) < 5 * 1024 * 1024:
                        return _err(400, "EntityTooSmall", f"part {n}", key)
                    datas.append(got[0])
                    md5s += bytes.fromhex(got[1])
                data = b"".join(datas)
                etag = f"{hashlib.md5(md5s).hexdigest()}-{len(want)}"
                objs[key] = StoredObject(data, etag, content_type=up.content_type, meta=up.meta)
                del ups[q["uploadId"]]
                return _xml(f'<CompleteMultipartUploadResult xmlns="{XMLNS}"><Bucket>{bucket}'
                            f"</Bucket><Key>{escape(key)}</Key><ETag>&quot;{etag}&quot;</ETag>"
                            "</CompleteMultipartUploadResult>")
        if m == "PUT" and req.headers.get("x-amz-copy-source"):      # CopyObject
            data = self._copy_source(req.headers["x-amz-copy-source"], None)
            if isinstance(data, web.Response):
                return data
            etag = hashlib.md5(data).hexdigest()
            objs[key] = StoredObject(data, etag, content_type=req.headers.get(
                "Content-Type", "application/octet-stream"))
            self.server_copies += 1
            return _xml(f'<CopyObjectResult xmlns="{XMLNS}"><ETag>&quot;{etag}&quot;</ETag>'
                        "</CopyObjectResult>")
        if m == "PUT":
            etag = hashlib.md5(body).hexdigest()
            objs[key] = StoredObject(body, etag, content_type=req.headers.get(
                "Content-Type", "application/octet-stream"), meta=_user_meta(req.headers))
            return web.Response(status=200, headers={"ETag": f'"{etag}"'})
        o = objs.get(key)
        if m == "DELETE":
            objs.pop(key, None)
            return web.Response(status=204)
        if o is None:
            if m == "HEAD":
                return web.Response(status=404)
            return _err(404, "NoSuchKey", "The specified key does not exist.", key)
        hdrs = {"ETag": f'"{o.etag}"', "Last-Modified": time.strftime(
            "%a, %d %b %Y %H:%M:%S GMT", time.gmtime(o.mtime)), "Accept-Ranges": "bytes",
                **o.meta}
        im = req.headers.get("If-Match")
        if im and im != "*" and im.strip('"') != o.etag:        # S3 conditional GET / HEAD
            return _err(412, "PreconditionFailed", "At least one of the pre-conditions you "
                        "specified did not hold", key)
        if m == "HEAD":
            hdrs["Content-Length"] = str(len(o.data))
            return web.Response(status=200, headers=hdrs)
        if m == "GET":
            rng = req.headers.get("Range")
            if rng and rng.startswith("bytes="):
                a, _, b = rng[6:].partition("-")
                start = int(a) if a else max(0, len(o.data) - int(b))
                end = int(b) if (b and a) else len(o.data) - 1
                end = min(end, len(o.data) - 1)
                if start > end:
                    return _err(416, "InvalidRange", "", key)
                hdrs["Content-Range"] = f"bytes {start}-{end}/{len(o.data)}"
                return web.Response(status=206, body=o.data[start:end + 1], headers=hdrs)
            return web.Response(status=200, body=o.data, headers=hdrs,
                                content_type=o.content_type)
        return _err(405, "MethodNotAllowed", "", key)
