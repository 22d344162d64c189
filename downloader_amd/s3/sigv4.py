"""AWS Signature Version 4 for S3 (what minio-js does inside ``triton-core/minio``).

Canonical request (method, URI, query, headers, signed headers, payload hash) -> string to
sign -> HMAC-SHA256 chain over date/region/service. ``UNSIGNED-PAYLOAD`` lets a file body go
to the socket with ``sendfile`` without a hashing pass; otherwise the payload SHA-256 comes
from the native hasher.
"""
from __future__ import annotations

import datetime as _dt
import hashlib
import hmac
from typing import Dict, Iterable, List, Mapping, Optional, Sequence, Tuple
from urllib.parse import quote

EMPTY_SHA256 = "e3b0c44298fc1c149afbf4c8996fb92427ae41e4649b934ca495991b7852b855"
UNSIGNED = "UNSIGNED-PAYLOAD"
# aws-chunked body without chunk signatures, followed by trailing headers (the CRC32C)
STREAMING_TRAILER = "STREAMING-UNSIGNED-PAYLOAD-TRAILER"
ALGO = "AWS4-HMAC-SHA256"


def uri_encode(s: str, keep_slash: bool) -> str:
    return quote(s, safe="/-_.~" if keep_slash else "-_.~")


def canonical_query(params: Iterable[Tuple[str, str]]) -> str:
    enc = sorted((uri_encode(k, False), uri_encode(v, False)) for k, v in params)
    return "&".join(f"{k}={v}" for k, v in enc)


def amz_dates(now: Optional[_dt.datetime] = None) -> Tuple[str, str]:
    t = now or _dt.datetime.now(_dt.timezone.utc)
    return t.strftime("%Y%m%dT%H%M%SZ"), t.strftime("%Y%m%d")


def _hmac(key: bytes, msg: str) -> bytes:
    return hmac.new(key, msg.encode("utf-8"), hashlib.sha256).digest()


_key_cache: Dict[Tuple[str, str, str, str], bytes] = {}


def signing_key(secret: str, date: str, region: str, service: str = "s3") -> bytes:
    ck = (secret, date, region, service)
    k = _key_cache.get(ck)
    if k is None:
        k = _hmac(_hmac(_hmac(_hmac(("AWS4" + secret).encode(), date), region), service),
                  "aws4_request")
        if len(_key_cache) > 64:
            _key_cache.clear()
        _key_cache[ck] = k
    return k


def canonical_request(method: str, path: str, query: Sequence[Tuple[str, str]],
                      headers: Mapping[str, str], signed: List[str], payload_hash: str) -> str:
    ch = "".join(f"{h}:{' '.join(str(headers[h]).strip().split())}\n" for h in signed)
    return "\n".join([method, uri_encode(path, True), canonical_query(query), ch,
                      ";".join(signed), payload_hash])


def sign(method: str, path: str, query: Sequence[Tuple[str, str]], headers: Dict[str, str],
         access_key: str, secret_key: str, region: str, payload_hash: str,
         now: Optional[_dt.datetime] = None, service: str = "s3") -> Dict[str, str]:
    """Add ``x-amz-date``, ``x-amz-content-sha256`` and ``Authorization`` to ``headers``
    (lower-case names; must already contain ``host``). Returns the same dict."""
    amzdate, date = amz_dates(now)
    headers["x-amz-date"] = amzdate
    headers["x-amz-content-sha256"] = payload_hash
    signed = sorted(headers.keys())
    creq = canonical_request(method, path, query, headers, signed, payload_hash)
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join([ALGO, amzdate, scope, hashlib.sha256(creq.encode()).hexdigest()])
    sig = hmac.new(signing_key(secret_key, date, region, service), sts.encode(),
                   hashlib.sha256).hexdigest()
    headers["authorization"] = (f"{ALGO} Credential={access_key}/{scope}, "
                                f"SignedHeaders={';'.join(signed)}, Signature={sig}")
    return headers


def presign(method: str, host: str, path: str, query: Sequence[Tuple[str, str]],
            access_key: str, secret_key: str, region: str, expires: int = 3600,
            now: Optional[_dt.datetime] = None, session_token: str = "",
            service: str = "s3") -> List[Tuple[str, str]]:
    """Query-string authentication (a presigned URL): returns ``query`` plus the X-Amz-*
    parameters, X-Amz-Signature last. Only ``host`` is signed and the payload is
    UNSIGNED-PAYLOAD, so the URL works for Range GETs and through any HTTP client."""
    amzdate, date = amz_dates(now)
    scope = f"{date}/{region}/{service}/aws4_request"
    q = list(query) + [("X-Amz-Algorithm", ALGO),
                       ("X-Amz-Credential", f"{access_key}/{scope}"),
                       ("X-Amz-Date", amzdate), ("X-Amz-Expires", str(int(expires))),
                       ("X-Amz-SignedHeaders", "host")]
    if session_token:
        q.append(("X-Amz-Security-Token", session_token))
    creq = canonical_request(method, path, q, {"host": host}, ["host"], UNSIGNED)
    sts = "\n".join([ALGO, amzdate, scope, hashlib.sha256(creq.encode()).hexdigest()])
    sig = hmac.new(signing_key(secret_key, date, region, service), sts.encode(),
                   hashlib.sha256).hexdigest()
    return q + [("X-Amz-Signature", sig)]


def verify_presigned(method: str, path: str, query: Sequence[Tuple[str, str]],
                     headers: Mapping[str, str], secrets: Mapping[str, str],
                     now: Optional[_dt.datetime] = None,
                     service: str = "s3") -> Tuple[bool, str]:
    """Server-side check of a presigned request (FakeS3). ``headers`` lower-cased."""
    q = dict(query)
    try:
        given = q["X-Amz-Signature"]
        access, date, region = q["X-Amz-Credential"].split("/")[:3]
        amzdate = q["X-Amz-Date"]
        expires = int(q["X-Amz-Expires"])
        signed = q["X-Amz-SignedHeaders"].split(";")
        t0 = _dt.datetime.strptime(amzdate, "%Y%m%dT%H%M%SZ").replace(tzinfo=_dt.timezone.utc)
    except (KeyError, ValueError):
        return False, "AuthorizationQueryParametersError"
    secret = secrets.get(access)
    if secret is None:
        return False, "InvalidAccessKeyId"
    if (now or _dt.datetime.now(_dt.timezone.utc)) > t0 + _dt.timedelta(seconds=expires):
        return False, "AccessDenied"                     # "Request has expired"
    rest = [(k, v) for k, v in query if k != "X-Amz-Signature"]
    try:
        creq = canonical_request(method, path, rest, headers, signed, UNSIGNED)
    except KeyError:
        return False, "AuthorizationQueryParametersError"
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join([ALGO, amzdate, scope, hashlib.sha256(creq.encode()).hexdigest()])
    want = hmac.new(signing_key(secret, date, region, service), sts.encode(),
                    hashlib.sha256).hexdigest()
    if not hmac.compare_digest(want, given):
        return False, "SignatureDoesNotMatch"
    return True, ""


def parse_authorization(value: str) -> Dict[str, str]:
    if not value.startswith(ALGO + " "):
        raise ValueError("not a SigV4 authorization header")
    out: Dict[str, str] = {}
    for part in value[len(ALGO) + 1:].split(","):
        k, _, v = part.strip().partition("=")
        out[k] = v
    return out


def verify(method: str, path: str, query: Sequence[Tuple[str, str]], headers: Mapping[str, str],
           secrets: Mapping[str, str], service: str = "s3") -> Tuple[bool, str]:
    """Server-side check (FakeS3). ``headers`` lower-cased. Returns (ok, reason)."""
    try:
        auth = parse_authorization(headers.get("authorization", ""))
        cred = auth["Credential"].split("/")
        access, date, region = cred[0], cred[1], cred[2]
        signed = auth["SignedHeaders"].split(";")
        given = auth["Signature"]
    except (ValueError, KeyError, IndexError):
        return False, "AuthorizationHeaderMalformed"
    secret = secrets.get(access)
    if secret is None:
        return False, "InvalidAccessKeyId"
    amzdate = headers.get("x-amz-date", "")
    payload_hash = headers.get("x-amz-content-sha256", "")
    try:
        creq = canonical_request(method, path, query, headers, signed, payload_hash)
    except KeyError:
        return False, "AuthorizationHeaderMalformed"
    scope = f"{date}/{region}/{service}/aws4_request"
    sts = "\n".join([ALGO, amzdate, scope, hashlib.sha256(creq.encode()).hexdigest()])
    want = hmac.new(signing_key(secret, date, region, service), sts.encode(),
                    hashlib.sha256).hexdigest()
    if not hmac.compare_digest(want, given):
        return False, "SignatureDoesNotMatch"
    return True, ""
